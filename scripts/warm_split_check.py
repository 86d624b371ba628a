import sys, numpy as np, time
sys.path[:0]=['tests','torj.jl_amd','oracle']
import torj_hip as T
from torj_hip import synthetic as S
from test_gpu_split import _fan, _run
eq=S.circular_tokamak(); hp=T.Plasma(*S.plasma_args(eq)); T.abs_Al_init(24)
for model, nr in ((2, 14), (3, 5)):
    pos,xp,Np,s0,w,om=_fan(T,hp,n_rings=nr)
    kw=dict(ds=1e-4,n_steps=2000,weights=w,traj_stride=100,absorption=model,psi_grid=np.linspace(0,1,500),deposition="reference",x_launch=pos,s0=s0)
    t=time.time(); a=_run(T,hp,1,0,xp,Np,om,1,**kw); ta=time.time()-t
    t=time.time(); b=_run(T,hp,3,0,xp,Np,om,1,**kw); tb=time.time()-t
    ex=np.abs(a.state[:,:6]-b.state[:,:6]).max()/np.abs(a.state[:,:6]).max()
    et=np.abs(a.state[:,6]-b.state[:,6])/np.maximum(np.abs(a.state[:,6]),1e-300)
    print(model, len(w), "status eq", np.array_equal(a.status,b.status), "steps eq", np.array_equal(a.steps,b.steps), "x/N %.2e"%ex, "tau max rel %.2e"%et.max(), "p99 %.2e"%np.quantile(et,0.99), "tau range %.3g-%.3g"%(a.state[:,6].min(),a.state[:,6].max()), "Pdep max abs %.2e"%np.abs(a.P_dep-b.P_dep).max(), "t fused %.1f split %.1f"%(ta,tb))
