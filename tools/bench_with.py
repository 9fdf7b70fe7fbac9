"""Run bench.py with module constants overridden (A/B runs without environment knobs):
    python tools/bench_with.py kernels.WGRAD_XPLANES=0 [-- bench args]"""
import importlib
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
args = sys.argv[1:]
rest = args[args.index("--") + 1:] if "--" in args else []
for a in (args[: args.index("--")] if "--" in args else args):
    name, val = a.split("=", 1)
    mod, attr = name.rsplit(".", 1)
    m = importlib.import_module("espnet_slurp_amd." + mod)
    setattr(m, attr, type(getattr(m, attr))(int(val)) if val.isdigit() else val)
    print(f"# {name} = {getattr(m, attr)!r}", file=sys.stderr)
sys.argv = [os.path.join(ROOT, "bench.py")] + rest
runpy.run_path(sys.argv[0], run_name="__main__")
