"""Scan of viscosity model variants against the simple and CONV goldens (dev-container study; reads
the goldens under tests/golden and runs the CPU oracle).  Omega22*: Neufeld correlation or the
Hirschfelder Lennard-Jones table with 3-point interpolation; fits: interval end, spacing, points."""
import json, numpy as np, sys
sys.path.insert(0,'.'); sys.path.insert(0,'tests')
from pychemkin_amd.mechanism import Mechanism
from oracle import transport_ref as tr
from oracle.oracle import Oracle
from conftest import ch4_air_Y, P_ATM
m = Mechanism.from_files('data/grimech30_chem.inp','data/grimech30_thermo.dat')
tp = tr.parse_transport(open('data/grimech30_transport.dat').read())
params = [tp[s.upper()] for s in m.species]
TS = np.array([0.1,0.2,0.3,0.4,0.5,0.6,0.7,0.8,0.9,1.0,1.2,1.4,1.6,1.8,2.0,2.5,3.0,3.5,4.0,5.0,6.0,7.0,8.0,9.0,10.,12.,14.,16.,18.,20.,25.,30.,35.,40.,50.,75.,100.])
O22 = np.array([4.1005,3.2626,2.8399,2.5310,2.2837,2.0838,1.9220,1.7902,1.6823,1.5929,1.4551,1.3551,1.2800,1.2219,1.1757,1.0933,1.0388,0.99963,0.96988,0.92676,0.89616,0.87272,0.85379,0.83795,0.82435,0.80184,0.78363,0.76834,0.75518,0.74364,0.71982,0.70097,0.68545,0.67232,0.65099,0.61397,0.58870])
def om_table(t):
    t = np.atleast_1d(t); out = np.empty_like(t)
    for i,x in enumerate(t):
        j = np.searchsorted(TS, x); j = min(max(j-1,1), len(TS)-2)
        xs, ys = TS[j-1:j+2], O22[j-1:j+2]
        # quadratic through 3 points
        out[i] = sum(ys[a]*np.prod([(x-xs[b])/(xs[a]-xs[b]) for b in range(3) if b!=a]) for a in range(3))
    return out
def eta_exact(T, omfun, polar=True):
    T=np.atleast_1d(T)
    eps=np.array([p[1] for p in params]); sig=np.array([p[2] for p in params])*1e-8; mu=np.array([p[3] for p in params])*1e-18
    ds = 0.5*mu*mu/(eps*1.380649e-16*sig**3)
    mm = m.wt/6.02214076e23
    ts = T[:,None]/eps[None,:]
    om = omfun(ts.ravel()).reshape(ts.shape) + (0.2*ds**2/ts if polar else 0)
    return (5/16)*np.sqrt(np.pi*mm*1.380649e-16*T[:,None])/(np.pi*sig**2*om)
neuf = lambda t: tr.omega22(t, 0.0)
def fit(omfun, tl, th, npts=50, logspace=False):
    Tf = np.exp(np.linspace(np.log(tl),np.log(th),npts)) if logspace else np.linspace(tl, th, npts)
    V = np.vander(np.log(Tf), 4, increasing=True)
    y = np.log(eta_exact(Tf, omfun))
    c,*_ = np.linalg.lstsq(V,y,rcond=None); return c.T
def mix(T, X, eta):
    X=np.atleast_2d(X); W=m.wt
    A=(1+W[:,None]/W[None,:])**-0.5/np.sqrt(8); B=(W[None,:]/W[:,None])**0.25
    s=np.sqrt(eta); phi=A[None]*(1+(s[:,:,None]/s[:,None,:])*B[None])**2
    return np.sum(X*eta/np.einsum('nkj,nj->nk',phi,X),axis=1)
g=json.load(open('tests/golden/simple.json')); Xs=np.asarray(g['species-mole_fraction'])
gc=json.load(open('tests/golden/CONV.json'))
orc=Oracle(m); Y0=ch4_air_Y(m,0.7)[0]
res,_,(ts,ys,ps,vs)=orc.reactor(800.0,3*P_ATM,10.0,Y0,t_save=np.asarray(gc['state-time']),problem=2,energy=1,t_end=0.1,atol=1e-10,rtol=1e-8,nneg=True,ign_mode='TIFP',profile=([0.0,0.01,2.0],[10.0,4.0,4.0]))
Tc=ys[:,0]; Xc=tr.mole_fractions(ys[:,1:], m.wt); gv=np.asarray(gc['state-viscocity'])
def report(label, etafun):
    s = mix([300.],Xs[None],etafun(np.array([300.])))[0]*100/g['state-viscosity'][0]-1
    c = mix(Tc,Xc,etafun(Tc))/gv-1
    print(f'{label:28s} simple {s:+.2e}  conv800 {c[0]:+.2e} 1061 {c[1]:+.2e} 1070 {c[3]:+.2e} burned {c[4]:+.2e}')
report('exact neufeld', lambda T: eta_exact(T, neuf))
report('exact table', lambda T: eta_exact(T, om_table))
for omn,omf in (('neuf',neuf),('table',om_table)):
    for th in (2500.,3000.,3500.,4000.,5000.,6000.):
        for lg in (False,True):
            f = fit(omf, 300., th, logspace=lg)
            report(f'fit {omn} {th} {"log" if lg else "lin"}', lambda T: np.exp(np.vander(np.log(T),4,increasing=True)@f.T))
print('---')
for th in (2700., 2900., 3000., 3100., 3300.):
    for npts in (20, 50, 100):
        f = fit(neuf, 300., th, npts=npts, logspace=True)
        report(f'neuf log {th} n{npts}', lambda T: np.exp(np.vander(np.log(T),4,increasing=True)@f.T))
