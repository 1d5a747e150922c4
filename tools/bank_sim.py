"""LDS bank-conflict model of the balanced CG SpMV gathers on the FullySup graph (diagnostic, CPU).

Builds the FullySup-shape kNN graph (exact float64 brute force), cuts each U row into virtual rows of 8
entries as row_build does, deals them to 512 threads (v = j * 512 + tid) and prices every
ds_read_b32 gather instruction by the guide's banking rule (2 groups of 32 lanes, bank =
(addr/4) mod 32, distinct addresses on one bank serialise, equal addresses broadcast).
Compares the stored order, a greedy per-wave reordering of each virtual row's 8 entries, and
row renumberings (RCM, random projection, class).   python tools/bank_sim.py
"""
import numpy as np, sys
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from graphlearninglayer_amd.synth import CONFIGS, synth
c=CONFIGS["fullysup"]
X,lab=synth(c["base"],c["batch"],c["d"],r=c["r"],seed=0)
# exact kNN (float64 brute force) and the symmetric union pattern, as the GPU builds it
Xd=X.astype(np.float64); sq=(Xd*Xd).sum(1)
D=sq[:,None]+sq[None,:]-2*Xd@Xd.T
np.fill_diagonal(D,-1.0)
ind=np.argsort(D,axis=1,kind="stable")[:,:c["k"]]
n=X.shape[0]
pairs=set()
for i in range(n):
    for j in ind[i,1:]:
        pairs.add((i,int(j))); pairs.add((int(j),i))
class _G: pass
g=_G(); pr=sorted(pairs); g.rows=np.array([a for a,_ in pr]); g.cols=np.array([b for _,b in pr])
base=c["base"]; m=c["batch"]
rows=[[] for _ in range(m)]
for r_,c_ in zip(g.rows,g.cols):
    if r_>=base and c_>=base: rows[r_-base].append(c_-base)
vr=[]
for u in range(m):
    L=rows[u]
    for j in range(0,len(L),8): vr.append(L[j:j+8])
V=len(vr); print("V",V)
def cost(instr_cols):
    # instr_cols: list of 64 col or None; cost = sum over groups max distinct-address multiplicity per bank
    t=0
    for g0 in (0,32):
        banks={}
        for cc in instr_cols[g0:g0+32]:
            if cc is None: continue
            banks.setdefault(cc%32,set()).add(cc)
        t+= max([len(s) for s in banks.values()]+[1])
    return t
def simulate(NT,RV,assign,greedy):
    total=0; ninstr=0
    for w in range(NT//64):
        for j in range(RV):
            lanes=[]
            for l in range(64):
                t=w*64+l
                v = t*RV+j if assign=="contig" else j*NT+t
                lanes.append(list(vr[v]) if v<V else [])
            if all(len(x)==0 for x in lanes): continue
            K=max(len(x) for x in lanes)
            if not greedy:
                for k in range(K):
                    total+=cost([x[k] if k<len(x) else None for x in lanes]); ninstr+=1
            else:
                rem=[list(x) for x in lanes]
                for k in range(K):
                    instr=[None]*64
                    for g0 in (0,32):
                        used={}
                        # lanes with more remaining first
                        order=sorted(range(g0,g0+32),key=lambda l:-len(rem[l]))
                        for l in order:
                            if not rem[l]: continue
                            # must place one if remaining == K-k (forced)
                            best=None
                            for idx,cc in enumerate(rem[l]):
                                b=cc%32
                                if b not in used or cc in used[b]: best=idx;break
                            if best is None:
                                if len(rem[l])>=K-k: best=min(range(len(rem[l])),key=lambda i:len(used.get(rem[l][i]%32,())))
                                else: continue
                            cc=rem[l].pop(best); instr[l]=cc; used.setdefault(cc%32,set()).add(cc)
                    total+=cost(instr); ninstr+=1
    return total, ninstr
for NT,RV in ((512,10),):
    for assign in ("contig","inter"):
        for gr in (False,True):
            t,n=simulate(NT,RV,assign,gr)
            print(NT,RV,assign,"greedy" if gr else "plain","cycles",t,"instr",n, "cyc/instr %.2f"%(t/n))

import scipy.sparse as sp
from scipy.sparse.csgraph import reverse_cuthill_mckee
A=sp.csr_matrix((np.ones(sum(len(r) for r in rows)),(np.repeat(np.arange(m),[len(r) for r in rows]),np.concatenate(rows))),shape=(m,m))
def sim_perm(perm,label):
    inv=np.empty(m,int); inv[perm]=np.arange(m)
    global vr,V
    vr=[]
    for newu in range(m):
        u=perm[newu]
        L=sorted(inv[c] for c in rows[u])
        for j in range(0,len(L),8): vr.append(L[j:j+8])
    V=len(vr)
    t,n=simulate(512,10,"inter",False)
    print(label,"cycles",t,"instr",n,"cyc/instr %.2f"%(t/n))
sim_perm(np.arange(m),"identity")
sim_perm(np.asarray(reverse_cuthill_mckee(A,symmetric_mode=True)),"rcm")
Xu=X[base:].astype(np.float64)
rp=np.random.default_rng(0).standard_normal(Xu.shape[1])
sim_perm(np.argsort(Xu@rp),"randproj")
# label-sorted (cluster) ordering by nearest... use class labels of the synthetic mixture as a proxy
sim_perm(np.argsort(lab[base:],kind="stable"),"class")

def simulate_diag(NT,RV,shift_fn):
    total=0; ninstr=0
    for w in range(NT//64):
        for j in range(RV):
            lanes=[]
            for l in range(64):
                t=w*64+l
                v = j*NT+t
                e=list(vr[v]) if v<V else []
                e=sorted(e,key=lambda cc: ((cc%32)-shift_fn(l))%32)
                lanes.append(e)
            if all(len(x)==0 for x in lanes): continue
            K=max(len(x) for x in lanes)
            for k in range(K):
                total+=cost([x[k] if k<len(x) else None for x in lanes]); ninstr+=1
    return total,ninstr
sim_perm(np.arange(m),"identity again")
for nm,f in (("l",lambda l:l%32),("0",lambda l:0),("2l",lambda l:(2*l)%32)):
    t,n=simulate_diag(512,10,f); print("diag",nm,t,n,"%.2f"%(t/n))
