import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rs-bann_amd"))
sys.argv=['bench.py','--no-cpu-baseline']
import bench
orig_perf=time.perf_counter
from bann import context as C
cls=C.BannContext
def wrap(name):
    f=getattr(cls,name)
    def g(self,*a,**k):
        t=orig_perf(); r=f(self,*a,**k); print(f"[t] {name} {1e3*(orig_perf()-t):.2f} ms", file=sys.stderr); return r
    setattr(cls,name,g)
for n in ["leapfrog_steps","leapfrog_end","residual_delta","synchronize","leapfrog_begin"]: wrap(n)
bench.main()
