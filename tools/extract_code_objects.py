"""Extract the gfx950 code objects from libsiren_mri_amd.so (its .hip_fatbin section holds one clang
offload bundle per translation unit) and disassemble them, for the static hazard checks
(tools/check_store_hazard.py, tools/check_lds_hazard.py).

    python tools/extract_code_objects.py [lib.so] [outdir]   -> outdir/tu<i>.co, outdir/tu<i>.dis
"""
import os
import struct
import subprocess
import sys

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
LLVM = "/opt/rocm/lib/llvm/bin"


def fatbin_section(path):
    """Bytes of the .hip_fatbin section (ELF64 little endian section table walk)."""
    data = open(path, "rb").read()
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    def sh(i):
        return struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize)
    stroff = sh(shstrndx)[4]
    for i in range(shnum):
        name_off, _, _, _, off, size = sh(i)[:6]
        end = data.index(b"\0", stroff + name_off)
        if data[stroff + name_off:end] == b".hip_fatbin":
            return data[off:off + size]
    raise RuntimeError(".hip_fatbin not found in " + path)


def code_objects(sec, arch="gfx950"):
    """The arch's code object of every offload bundle in the section."""
    out, pos = [], 0
    while True:
        pos = sec.find(MAGIC, pos)
        if pos < 0:
            return out
        n, = struct.unpack_from("<Q", sec, pos + len(MAGIC))
        p = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", sec, p)
            triple = sec[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if arch in triple:
                out.append(sec[pos + off:pos + off + size])
        pos = p


def extract(lib, outdir):
    os.makedirs(outdir, exist_ok=True)
    paths = []
    for i, co in enumerate(code_objects(fatbin_section(lib))):
        p = os.path.join(outdir, f"tu{i}.co")
        open(p, "wb").write(co)
        dis = p[:-3] + ".dis"
        with open(dis, "w") as f:
            subprocess.check_call([os.path.join(LLVM, "llvm-objdump"), "-d", p], stdout=f)
        paths.append(dis)
    return paths


if __name__ == "__main__":
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(root, "siren_mri_amd", "libsiren_mri_amd.so")
    outdir = sys.argv[2] if len(sys.argv) > 2 else "/tmp/siren_co"
    for p in extract(lib, outdir):
        print(p)
