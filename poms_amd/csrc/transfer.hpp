// The fused residual -> restriction pass descriptor (transfer.hip, poms_abi.hip).
#pragma once
#include "common.hpp"

namespace poms {

// One pass of the fused residual -> restriction: up to 3 inputs and 3 outputs
// sharing one AxisPass geometry; m[o][k] (device, rows padded to the pass's ncm
// columns, null = no term) maps input k into output o.
struct MultiPass {
    AxisPass ps;
    const double* in[3];
    double* out[3];
    const double* m[3][3];
    int ni, no;
};

int mrestrict_launch(int ncm, const MultiPass& mp, double* part, hipStream_t st);
int64_t mrestrict_scratch(const MultiPass& mp, int ncm);

}  // namespace poms
