# Estimate (host, timing-free) of what direction-bin culling of Voronoi neighbour entries would save: a
# 1e5-site Plummer tessellation (scipy qhull), per-bin kept entries and the expected groups of 4 per wave
# of 64 rays ("Voronoi walk", round 4). usage: python3 tools/vor_cull_estimate.py
import numpy as np
from scipy.spatial import Voronoi
rng=np.random.default_rng(1)
N=100000
# Plummer positions
u=rng.random(N); r=1/np.sqrt(u**(-2/3)-1); r=np.minimum(r,20)
v=rng.normal(size=(N,3)); v/=np.linalg.norm(v,axis=1)[:,None]; P=v*r[:,None]
vor=Voronoi(P)
nb=[[] for _ in range(N)]
for a,b in vor.ridge_points: nb[a].append(b); nb[b].append(a)
cnt=np.array([len(x) for x in nb])
print('mean neighbours %.2f max %d'%(cnt.mean(),cnt.max()))
def axes(kind):
    if kind==8: A=np.array([[sx,sy,sz] for sx in(-1,1) for sy in(-1,1) for sz in(-1,1)],float)
    elif kind==26: A=np.array([[x,y,z] for x in(-1,0,1) for y in(-1,0,1) for z in(-1,0,1) if (x,y,z)!=(0,0,0)],float)
    A/=np.linalg.norm(A,axis=1)[:,None]; return A
# covering radius by sampling directions
K=rng.normal(size=(200000,3)); K/=np.linalg.norm(K,axis=1)[:,None]
sample=rng.choice(N,20000,replace=False)
for B in (8,26):
    A=axes(B); dots=K@A.T; best=dots.argmax(1); ang=np.arccos(np.clip(dots.max(1),-1,1))
    th=np.array([ang[best==b].max() for b in range(B)])
    kept=[]
    for i in sample:
        n=P[nb[i]]-P[i]; n/=np.linalg.norm(n,axis=1)[:,None]
        b=rng.integers(B)  # a ray's bin
        a=A[b]; ang_n=np.arccos(np.clip(n@a,-1,1))
        kept.append(int((ang_n < np.pi/2+th[b]+1e-3).sum()))
    kept=np.array(kept); full=cnt[sample]
    def wmax(x): 
        m=[x[rng.integers(len(x),size=64)].max() for _ in range(4000)]; return np.mean(m)
    groups=lambda x: np.mean([int(np.ceil(x[rng.integers(len(x),size=64)].max()/4)) for _ in range(4000)])
    print('B=%d cone half-angles max %.1f deg; kept mean %.2f of %.2f; wave-max %.1f vs %.1f; groups %.2f vs %.2f'%(B,np.degrees(th.max()),kept.mean(),full.mean(),wmax(kept),wmax(full),groups(kept),groups(full)))
