"""Offline estimate of the hub index's effect on config #4's nesting graph (CPU only, numpy).

Rebuilds the generator's group nesting (keto_amd/csrc/synth.cpp ks_social_generate: Zipf
popularity on both ends of each parent edge, acyclic by a random topological order, one
edge per group) for G groups, marks the H groups with the most children as hubs, and
reports, for 200 roots (half Zipf-popular, half uniform), the size of the search that stops
at hubs and the number of hubs it reaches.  Used to pick the hub rule (>= 8 interior
successors, see DESIGN.md "Config #4 and the hub index").

    python tools/hub_sim.py 1e7     # 10M groups = the 1B-tuple configuration
"""
import numpy as np, scipy.sparse as sp, sys, time
G=int(float(sys.argv[1])); rng=np.random.default_rng(1)
k=np.arange(1,G+1,dtype=np.float64); cdf=np.cumsum(1/k); cdf/=cdf[-1]
pop=rng.permutation(G); topo=rng.permutation(G)
n=G
a=pop[np.minimum(np.searchsorted(cdf,rng.random(n)),G-1)]; b=pop[np.minimum(np.searchsorted(cdf,rng.random(n)),G-1)]
m=a!=b; a,b=a[m],b[m]
sw=topo[a]>topo[b]; a2=np.where(sw,b,a); b2=np.where(sw,a,b)
A=sp.csr_matrix((np.ones(len(a2),np.int8),(a2,b2)),shape=(G,G))
deg=np.diff(A.indptr)
order=np.argsort(-deg,kind='stable')
roots=np.concatenate([pop[np.minimum(np.searchsorted(cdf,rng.random(100)),G-1)], rng.integers(0,G,100)])
for H in [0,1024,4096,16384,65536]:
    hub=np.zeros(G,bool); hub[order[:H]]=True
    print("H",H,"max nonhub deg",deg[order[H]] if H<G else 0, end=" ")
    sizes=[];hubs=[]
    t=time.time()
    for r in roots:
        vis=np.zeros(G,bool); reached=np.zeros(G,bool)
        fr=np.array([r]) if not hub[r] else np.array([],int)
        if hub[r]: reached[r]=True
        while len(fr):
            nb=A[fr].indices
            nb=np.unique(nb); nb=nb[~vis[nb]]; vis[nb]=True
            reached[nb[hub[nb]]]=True
            fr=nb[~hub[nb]]
        sizes.append(vis.sum()); hubs.append(reached.sum())
    s=np.array(sizes); h=np.array(hubs)
    print("closure mean %.0f p50 %d p99 %d max %d | hubs reached mean %.0f max %d  (%.1fs)"%(s.mean(),np.median(s),np.percentile(s,99),s.max(),h.mean(),h.max(),time.time()-t),flush=True)
