"""Per-kernel register / spill / LDS table of the native library (hipcc resource-usage remarks).

    python tools/resource_usage.py [filter]
"""
import re
import subprocess
import sys

SRCS = ("siren_mri_amd/csrc/siren_runtime.hip", "siren_mri_amd/csrc/siren_fwdreg_inst.hip")
out = ""
for src in SRCS:
    cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", "-o", "/tmp/_ru.o", src,
           "-Rpass-analysis=kernel-resource-usage"]
    out += subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    txt = m.group(1).strip()
    if txt.startswith("Function Name:"):
        cur = {"name": txt.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in txt:
        k, v = txt.split(":", 1)
        cur[k.strip()] = v.strip()
flt = sys.argv[1] if len(sys.argv) > 1 else ""
demangle = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                          text=True).stdout.splitlines()
print(f"{'kernel':70s} {'VGPR':>5s} {'AGPR':>5s} {'vspill':>6s} {'sspill':>6s} {'LDS':>7s} {'occ':>4s}")
for r, dn in zip(rows, demangle):
    if flt not in dn:
        continue
    dn = dn.replace("siren::", "").replace("(siren::", "(")
    print(f"{dn[:70]:70s} {r.get('VGPRs', '?'):>5s} {r.get('AGPRs', '?'):>5s} {r.get('VGPRs Spill', '?'):>6s} "
          f"{r.get('SGPRs Spill', '?'):>6s} {r.get('LDS Size [bytes/block]', '?'):>7s} "
          f"{r.get('Occupancy [waves/SIMD]', '?'):>4s}")
