"""Each SVD route's own error against the exact SVD (the certificate study): the
Jacobi route's f64 factors (oracle svd_blocks_f64) and the dgesdd route's (orc_lp_svd_blocks_f64)
against a long-double refinement of LAPACK's (two Ogita-Aishima steps, 64-bit significands), in
units of 2^-53 sigma_1 / m_k per triplet (U, V columns) and of 2^-53 sigma_1 (sigma_k), over the
unflagged blocks of one 1080p frame.  usage: route_errors.py B noise|photo"""
import os
import sys

import numpy as np

_R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [_R, os.path.join(_R, 'tests'), os.path.join(_R, 'tools', 'exp')]
from cert_study import *
LD=np.longdouble
def refine(D, U, s, V, it=2):
    A = D.astype(LD); U=U.astype(LD); V=V.astype(LD); s=s.astype(LD)
    b=A.shape[1]; I=np.eye(b,dtype=LD)
    for _ in range(it):
        R = I - np.matmul(np.swapaxes(U,1,2),U); S = I - np.matmul(np.swapaxes(V,1,2),V)
        T = np.matmul(np.matmul(np.swapaxes(U,1,2),A),V)
        d = np.diagonal(T,axis1=1,axis2=2); rd=np.diagonal(R,axis1=1,axis2=2); sd=np.diagonal(S,axis1=1,axis2=2)
        s = d/(1-(rd+sd)/2)
        al = T + s[:,None,:]*R; be = np.swapaxes(T,1,2) + s[:,None,:]*S
        den = s[:,None,:]**2 - s[:,:,None]**2
        np.einsum('nii->ni',den)[:] = 1
        F = (al*s[:,None,:] + be*s[:,:,None])/den
        G = (al*s[:,:,None] + be*s[:,None,:])/den
        np.einsum('nii->ni',F)[:] = rd/2; np.einsum('nii->ni',G)[:] = sd/2
        U = U + np.matmul(U,F); V = V + np.matmul(V,G)
    return U,s,V
b=int(sys.argv[1]); kind=sys.argv[2]
H,W=1080,1920
cov = O.synth_bytes(0x5EED0001, 0, 1, H*W*3).reshape(H,W,3) if kind=='noise' else photo_cover(H,W,100)
D,(Uj,sj,Vj),(Ul,sl,Vl) = frame(cov,b)
m,s1,keep = gaps(sj)
ok = (s1>0) & ~((np.where(keep, s1[:,None]/np.where(m>0,m,np.inf),0).max(1))>2**20) & keep.all(1)
D,Uj,sj,Vj,Ul,sl,Vl,m,s1 = (a[ok] for a in (D,Uj,sj,Vj,Ul,sl,Vl,m,s1))
Ue,se,Ve = refine(D,Ul,sl,Vl)
def err(Ux,Vx,sx):
    sg = np.sign(np.einsum('nrk,nrk->nk',Ux.astype(LD),Ue)); sg[sg==0]=1
    du = np.abs(Ux - Ue*sg[:,None,:]).max(1); dv=np.abs(Vx-Ve*sg[:,None,:]).max(1)
    ek = EPS*s1[:,None]/m
    return (du/ek).astype(float), (dv/ek).astype(float), (np.abs(sx-se)/(EPS*s1[:,None])).astype(float)
for name,(U,s,V) in (('jacobi',(Uj,sj,Vj)),('lapack',(Ul,sl,Vl))):
    ru,rv,rs = err(U,V,s)
    print(name, 'u max %.2f q999 %.2f | v max %.2f q999 %.2f | s max %.2f' % (ru.max(), np.quantile(ru.max(1),.999), rv.max(), np.quantile(rv.max(1),.999), rs.max()))
# refinement self-consistency: refine from jacobi too
Ue2,se2,Ve2 = refine(D,Uj,sj,Vj)
sg = np.sign(np.einsum('nrk,nrk->nk',Ue2,Ue)); 
print('refine agreement', float((np.abs(Ue2-Ue*sg[:,None,:]).max(1)/(EPS*s1[:,None]/m)).max()))
