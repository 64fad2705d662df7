import runpy, sys
sys.path.insert(0, ".")
import pggan_amd._lib as L
lib = sys.argv[1]
if lib != "main":
    L.load_library.__defaults__ = (lib,)
sys.argv = ["kbench.py", "--iters", "30"] + sys.argv[2:]
runpy.run_path("tools/kbench.py", run_name="__main__")
