import cProfile, pstats, sys, os, io
sys.argv = ["bench.py", "--graphs", "off", "--steps", "12", "--warmup", "8"]
sys.path.insert(0, os.getcwd())
import runpy
pr = cProfile.Profile()
pr.enable()
try:
    runpy.run_path("bench.py", run_name="__main__")
finally:
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(35)
    open("gpurun_out/host_prof.txt", "w").write(s.getvalue())
