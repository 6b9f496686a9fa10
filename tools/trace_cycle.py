# One V-cycle of a rocprofv3 --kernel-trace csv (cycles split at the prolongation passes):
# span vs busy (union of kernel intervals) vs summed durations, per-queue kernel totals, and a
# window of the timeline.  python tools/trace_cycle.py run_kernel_trace.csv [offset]
import csv, collections, sys
r=list(csv.DictReader(open(sys.argv[1])))
r.sort(key=lambda x:int(x['Start_Timestamp']))
pro=[i for i,x in enumerate(r) if 'prolong_pass' in x['Kernel_Name']]
cyc=[(pro[3*k+2]) for k in range(len(pro)//3)]
a,b=cyc[1]+1,cyc[2]+1
seg=r[a:b]
S=int(seg[0]['Start_Timestamp']); E=int(seg[-1]['End_Timestamp'])
iv=sorted((int(x['Start_Timestamp']),int(x['End_Timestamp'])) for x in seg)
busy=0;cs,ce=iv[0]
for s,e in iv[1:]:
    if s>ce: busy+=ce-cs; cs,ce=s,e
    else: ce=max(ce,e)
busy+=ce-cs
tot=sum(e-s for s,e in iv)
print('cycle span ms',(E-S)/1e6,'busy',busy/1e6,'sum',tot/1e6, 'n',len(seg))
st=collections.defaultdict(lambda:[0,0])
for x in seg:
    k=x['Kernel_Name'][:60]; st[(x['Queue_Id'],k)][0]+=1; st[(x['Queue_Id'],k)][1]+=int(x['End_Timestamp'])-int(x['Start_Timestamp'])
for k,v in sorted(st.items(),key=lambda kv:-kv[1][1])[:12]: print(k, v[0], round(v[1]/1e6,2))
o=int(sys.argv[2]) if len(sys.argv)>2 else 700
seg2=seg[o:o+30]
T=int(seg2[0]['Start_Timestamp'])
for x in seg2:
    s=(int(x['Start_Timestamp'])-T)/1e3; e=(int(x['End_Timestamp'])-T)/1e3
    print(f"{s:9.1f} {e:9.1f} {e-s:7.1f} q{x['Queue_Id']} grid{int(x['Grid_Size_X'])//int(x['Workgroup_Size_X'])} {x['Kernel_Name'][:50]}")
