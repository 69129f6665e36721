import csv,glob,sys
from collections import defaultdict
f=glob.glob(sys.argv[1]+'/**/*kernel_trace.csv',recursive=True)[0]
rows=sorted(csv.DictReader(open(f)),key=lambda r:int(r["Start_Timestamp"]))
def short(n): return n.split("(")[0].replace("void ","").replace("kb::","")
rounds=[];cur=None;w=-1
for r in rows:
    k=short(r["Kernel_Name"]);a,b=int(r["Start_Timestamp"]),int(r["End_Timestamp"])
    if k=="k_alive_bits": cur=defaultdict(list);rounds.append(cur);w=-1
    if cur is None: continue
    if k in("k_route","k_route_x"): w+=1
    cur[w].append((k,(b-a)/1e3))
lo=int(sys.argv[2]); hi=int(sys.argv[3])
sel=rounds[lo:hi]
for wv in range(-1,9):
    agg=defaultdict(float)
    for rd in sel:
        for k,d in rd[wv]: agg[k]+=d
    tot=sum(agg.values())/len(sel)
    print(f"wave {wv} {tot:7.1f}us ", " ".join(f"{k}:{agg[k]/len(sel):.1f}" for k in agg if agg[k]/len(sel)>3))
