"""LDS bank model of k_normals_stile's stencil reads (grid.hip StileShape):
per 32-lane half-wave, distinct slots per bank (bank = slot mod 32 for
ds_read_b64 of (x, y) pairs and ds_read2_b32 of z) averaged over the
Stencil220 rows, with each lane's random per-axis mirroring; 1.0 = conflict
free.  Usage: python tools/stile_banks.py"""
import numpy as np, itertools
rows220=[(-2,-2,-1,3),(-1,-2,-2,5),(0,-2,-2,5),(1,-2,-2,5),(2,-2,-1,4),(-2,-1,-2,5),(-1,-1,-2,6),(0,-1,-2,6),(1,-1,-2,6),(2,-1,-2,5),(3,-1,-1,3),(-2,0,-2,5),(-1,0,-2,6),(0,0,-2,6),(1,0,-2,6),(2,0,-2,5),(3,0,-1,3),(-2,1,-2,5),(-1,1,-2,6),(0,1,-2,6),(1,1,-2,6),(2,1,-2,5),(3,1,-1,3),(-2,2,-1,4),(-1,2,-2,5),(0,2,-2,5),(1,2,-2,5),(2,2,-2,5),(-1,3,-1,3),(0,3,-1,3),(1,3,-1,3)]
rng=np.random.default_rng(0)
def sim(SY,SZ,lanemap,trials=200,mirror=True):
    tot=0; ideal=0
    for _ in range(trials):
        lx,ly,lz=lanemap
        qs=(lx+3)+SY*(ly+3)+SZ*(lz+3)
        if mirror:
            sx=rng.integers(0,2,64)*2-1; sy=rng.integers(0,2,64)*2-1; sz=rng.integers(0,2,64)*2-1
        else:
            sx=sy=sz=np.ones(64,int)
        for dy,dz,xa,ln in rows220:
            st=qs+dy*SY*sy+dz*SZ*sz+np.where(sx>0,xa,-(xa+ln-1))
            for i in range(ln):
                s=st+i
                for half in (s[:32],s[32:]):
                    u=np.unique(half)
                    b=u%32
                    tot+=np.bincount(b).max(); ideal+=1
    return tot/ideal
lane=np.arange(64); cur=(lane&3,(lane>>2)&3,lane>>4)
print("current 10/140 mirror", sim(10,140,cur))
print("current 10/140 no-mirror", sim(10,140,cur,mirror=False))
print("12/176 mirror", sim(12,176,cur))
print("12/176 no-mirror", sim(12,176,cur,mirror=False))
print("10/144 mirror", sim(10,144,cur))
res=[]
maps={"xyz":cur,"xzy":(lane&3,lane>>4,(lane>>2)&3)}
for SY in (10,11,12):
    for SZ in range(SY*14, 173):
        for mn,m in maps.items():
            if mn=="xzy": continue
            v=sim(SY,SZ,m,trials=20)
            res.append((v,SY,SZ,mn))
res.sort()
print(res[:12])
print("----")
maps2={
 "xyz": cur,
 "x,ylo,z|yhi": (lane&3, ((lane>>2)&1) | ((lane>>5)<<1), (lane>>3)&3),
 "x,y,z-even|odd": (lane&3, (lane>>2)&3, ((lane>>4)&1)*2 + (lane>>5)),
}
for SZ in (140,144,148,150,152,156):
    for mn,m in maps2.items():
        print(SZ, mn, round(sim(10,SZ,m,trials=40),3))
