"""cProfile of the host side of bench.py steps (which Python / ctypes calls the enqueue
time goes to).  python tools/host_profile.py out.pstats  (then pstats on the box)"""
import cProfile
import pstats
import sys

sys.argv = ["bench.py", "--steps", "3", "--warmup", "2", "--no-timer", "--no-cpu-baseline", "--no-prefetch"]
import runpy  # noqa: E402

pr = cProfile.Profile()
pr.enable()
try:
    runpy.run_path("bench.py", run_name="__main__")
finally:
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)
