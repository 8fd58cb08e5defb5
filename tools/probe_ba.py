import sys, time, random
import os; R=os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0,R+'/structure-from-motion-_amd'); sys.path.insert(0,R+'/oracle')
import numpy as np, _sfmcore as c, sfm_synthetic as syn
print("devices", c.device_count())
x1,x2,idx,_=syn.two_view(seed=0)
random.seed(0); s=c.sample_table(5000,8,16384)
for i in range(3):
    t=time.perf_counter(); b,F,m,cnt=c.ransac_f8(x1,x2,s,0.06,want_counts=True); dt=time.perf_counter()-t
    print("ransac", b, m.sum(), f"{dt*1e3:.2f} ms", "timings", c.last_timings().round(4))
for name in ("cfg3","cfg4","cfg5"):
    t=time.perf_counter(); p=syn.ba_problem_cfg(name, dense=False); tg=time.perf_counter()-t
    cams0=np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    t=time.perf_counter()
    prob=c.BAProblem(cams0,p["X0"],p["cam_idx"],p["pt_idx"],p["obs"],syn.K_REF)
    prob.set_timing()
    tc=time.perf_counter()-t
    rep=prob.solve(max_iterations=30)
    n=len(p["cam_idx"])
    print(name, f"gen {tg:.1f}s create {tc:.2f}s", {k:(round(v,4) if isinstance(v,float) else v) for k,v in rep.items()}, "rmse", syn.rmse_from_cost(rep["cost0"],n), "->", syn.rmse_from_cost(rep["cost"],n))
    print("  kernel ms/iter", {k:round(v,4) for k,v in prob.kernel_times().items()})
    prob.reset(); rep=prob.solve(max_iterations=10, fixed_iterations=True)
    print("  fixed10", rep["iterations"], f"{rep['t_loop_ms']:.2f} ms -> {rep['t_loop_ms']/10:.3f} ms/iter", {k:round(v,4) for k,v in prob.kernel_times().items()})
    prob.close()
