// Shared by poms_abi.hip (op_run_split) and comm.hip (poms_op_run_dist).
#pragma once

namespace poms {

// Ordering hooks of a split operator call (op_run_split): the boundary launch goes
// to `bstream` (nullptr: the caller's stream) after ghosts_on(arg, its stream) made
// that stream wait for the ghost exchange; join(arg, from, to) makes `to` wait for
// the work queued on `from`.
struct SplitHooks {
    void* bstream;
    int (*ghosts_on)(void* arg, void* stream);
    int (*join)(void* arg, void* from, void* to);
    void* arg;
};

}  // namespace poms
