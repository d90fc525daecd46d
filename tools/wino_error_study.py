"""fp32 error of Winograd F(m×m, 3×3) against the direct conv (numpy), for choosing the F(4×4) points.

    python tools/wino_error_study.py > profiles/r2/wino_error_study.txt

Builds Aᵀ, G, Bᵀ for any interpolation points (Cook-Toom / Lavin construction, exact fractions), checks the
1-D identity, then runs a 24×24×256 → 64 conv on relu-like activations in fp32 (transforms, GEMM and
inverse transform all rounded to fp32, U = G g Gᵀ in fp64) and reports max |e| / Σ|a||b| and rms error
against an fp64 direct conv, next to the fp32 direct conv. The chosen F(4×4) points (0, -1, 1, ½, -2, ∞)
are the ones winograd.hip / ops.WINO_* use.
"""
import numpy as np
from fractions import Fraction as Fr
def mats(m, r, pts):
    a = m + r - 1
    pts=[Fr(p) for p in pts]
    assert len(pts)==a-1
    AT=[[p**i for p in pts]+[Fr(1) if i==m-1 else Fr(0)] for i in range(m)]
    G=[]
    for j,pj in enumerate(pts):
        f=Fr(1)
        for i,pi in enumerate(pts):
            if i!=j: f*= (pj-pi)
        G.append([pj**k/f for k in range(r)])
    G.append([Fr(0)]*(r-1)+[Fr(1)])
    # BT rows: coefficients of M_j(x) = prod_{i!=j}(x - p_i) (ascending), padded to length a; last: M(x)
    def polymul(p,q):
        out=[Fr(0)]*(len(p)+len(q)-1)
        for i,x in enumerate(p):
            for j,y in enumerate(q): out[i+j]+=x*y
        return out
    BT=[]
    for j in range(a-1):
        poly=[Fr(1)]
        for i,pi in enumerate(pts):
            if i!=j: poly=polymul(poly,[-pi,Fr(1)])
        BT.append(poly+[Fr(0)]*(a-len(poly)))
    poly=[Fr(1)]
    for pi in pts: poly=polymul(poly,[-pi,Fr(1)])
    BT.append(poly+[Fr(0)]*(a-len(poly)))
    f=lambda M: np.array([[float(x) for x in row] for row in M])
    return f(AT), f(G), f(BT)
def check1d(m,r,pts):
    AT,G,BT=mats(m,r,pts)
    rng=np.random.default_rng(0); d=rng.standard_normal(m+r-1); g=rng.standard_normal(r)
    y=AT@((G@g)*(BT@d))
    ref=np.array([sum(d[i+k]*g[k] for k in range(r)) for i in range(m)])
    return np.abs(y-ref).max()
for pts in ([0,1,-1],[0,1,-1,2,-2],[0,1,-1,Fr(1,2),Fr(-1,2)]):
    m=len(pts)+1-3+1
    print(pts, m, check1d(m,3,pts))

def conv_direct(x,w):
    H,W,C=x.shape; xp=np.pad(x,((1,1),(1,1),(0,0)))
    out=np.zeros((H,W,w.shape[0]),dtype=x.dtype)
    for dy in range(3):
        for dx in range(3):
            out+= xp[dy:dy+H,dx:dx+W,:]@w[:,dy,dx,:].T
    return out
def wino2d(x,w,AT,G,BT,dt):
    m=AT.shape[0]; a=AT.shape[1]
    H,W,C=x.shape; Co=w.shape[0]
    th,tw=(H+m-1)//m,(W+m-1)//m
    xp=np.zeros((th*m+2,tw*m+2,C),dt); xp[1:H+1,1:W+1]=x
    U=np.einsum('ik,oklc,jl->ijoc',G,w.astype(np.float64),G).astype(dt)
    P=np.zeros((th,tw,a,a,C),dt)
    for i in range(a):
        for j in range(a):
            P[:,:,i,j]=xp[i:i+th*m:m, j:j+tw*m:m][:th,:tw]
    BTd=BT.astype(dt)
    V=np.einsum('ik,yxklc->yxilc',BTd,P).astype(dt)
    V=np.einsum('jl,yxilc->yxijc',BTd,V).astype(dt)
    Mm=np.einsum('yxijc,ijoc->yxijo',V,U).astype(dt)
    ATd=AT.astype(dt)
    Y=np.einsum('pi,yxijo->yxpjo',ATd,Mm).astype(dt)
    Y=np.einsum('qj,yxpjo->yxpqo',ATd,Y).astype(dt)
    return Y.transpose(0,2,1,3,4).reshape(th*m,tw*m,Co)[:H,:W]
rng=np.random.default_rng(0)
H=W=24; C=256; Co=64
x=np.maximum(rng.standard_normal((H,W,C)),0)*0.5+0.01*rng.standard_normal((H,W,C))
w=rng.standard_normal((Co,3,3,C))/np.sqrt(9*C)
ref=conv_direct(x,w); absref=conv_direct(np.abs(x),np.abs(w))
def rep(name,o):
    e=np.abs(o.astype(np.float64)-ref)
    print(f'{name:40s} max|e|/sum|ab| {(e/absref).max():.3g}  rms {np.sqrt((e**2).mean()/(ref**2).mean()):.3g}')
x32,w32=x.astype(np.float32),w.astype(np.float32)
rep('direct fp32',conv_direct(x32,w32))
for name,pts in (('F23 0,1,-1',[0,1,-1]),('F43 0,1,-1,2,-2',[0,1,-1,2,-2]),('F43 0,1,-1,1/2,-1/2',[0,1,-1,Fr(1,2),Fr(-1,2)]),('F43 0,-1,1,1/2,-2',[0,-1,1,Fr(1,2),-2]),('F63 0,1,-1,2,-2,1/2,-1/2',[0,1,-1,2,-2,Fr(1,2),Fr(-1,2)])):
    AT,G,BT=mats(len(pts)-1,3,pts)
    rep(name,wino2d(x32,w32,AT,G,BT,np.float32))
