import os, sys
sys.path.insert(0, os.getcwd())
exec(open("tools/psnr_ab.py").read().split("_native.load_library()")[0])
_native.load_library()
st = tuple(range(300, 801, 20))
print("steps", st)
print("fp32", run("fp32", steps=st), flush=True)
print("bf16", run("bf16", steps=st), flush=True)
