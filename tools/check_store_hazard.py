"""Static check of the store-hazard rule (siren_common.h) on a disassembled code object:
    llvm-objdump -d lib.co > lib.dis; python tools/check_store_hazard.py lib.dis [kernel-substring] [--all-operands]
For every buffer / scratch / global store in the matching kernels, report any instruction that writes one of the
store's data VGPRs (--all-operands: also its address VGPR and descriptor SGPRs) before an
s_waitcnt vmcnt(0), the only wait that guarantees the store has read them."""
import re
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
path = args[0]
filt = args[1] if len(args) > 1 else "fused_fwd_reg_kernel"
text = open(path).read().split("\n")
kernels = {}
cur = None
for line in text:
    m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
    if m:
        cur = m.group(1) if filt in m.group(1) else None
        if cur:
            kernels[cur] = []
        continue
    if cur and line.strip():
        ins = re.sub(r"^\s*[0-9a-f]+:\s+(?:[0-9a-f]{8} ?)+", "", line).split("//")[0].strip()
        if ins:
            kernels[cur].append(ins)


def regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def sregs(tok):
    m = re.match(r"s\[(\d+):(\d+)\]", tok)
    if m:
        return {("s", r) for r in range(int(m.group(1)), int(m.group(2)) + 1)}
    m = re.match(r"s(\d+)$", tok)
    return {("s", int(m.group(1)))} if m else set()


def operands(ins):
    """Registers a buffer store reads: data VGPRs, the address VGPR, the descriptor SGPRs."""
    ops = [t.strip() for t in ins.split(None, 1)[1].split(",")]
    out = set(regs(ops[0]))
    if len(ops) > 1:
        out |= regs(ops[1])
    if len(ops) > 2:
        out |= sregs(ops[2])
    return out


def swrites(ins):
    op = ins.split()[0]
    if not op.startswith("s_") or op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_cbranch", "s_branch",
                                                 "s_setprio", "s_sleep", "s_endpgm")):
        return set()
    toks = ins.split(None, 1)
    return sregs(toks[1].split(",")[0].strip()) if len(toks) > 1 else set()


def writes(ins):
    op = ins.split()[0]
    if op.startswith(("buffer_store", "global_store", "ds_write", "s_", "scratch_store", "global_load_lds",
                      "buffer_load_dword") ) and "lds" in ins:
        return set()
    if op.startswith(("buffer_store", "global_store", "ds_write", "s_", "scratch_store")):
        return set()
    toks = ins.split(None, 1)
    if len(toks) < 2:
        return set()
    return regs(toks[1].split(",")[0].strip())


bad = 0
nstores = 0
for k, body in kernels.items():
    for i, ins in enumerate(body):
        if not ins.startswith(("buffer_store", "scratch_store", "global_store")):
            continue
        nstores += 1
        first = ins.split(None, 1)[1].split(",")
        # buffer_store DATA, ADDR, SRD ...; scratch_store ADDR|off, DATA, ...; global_store ADDR, DATA, ...
        dtok = first[0].strip() if ins.startswith("buffer_store") else first[1].strip()
        data = operands(ins) if "--all-operands" in sys.argv and ins.startswith("buffer_store") else regs(dtok)
        for j in range(i + 1, len(body)):
            if re.match(r"s_waitcnt .*vmcnt\(0\)", body[j]) or body[j].startswith("s_endpgm"):
                break
            w = (writes(body[j]) | swrites(body[j])) & data
            if w:
                bad += 1
                print(f"{k[:60]} #{i}: {ins}  <- written {j - i} later by: {body[j]}")
                break
print(f"{len(kernels)} kernels, {nstores} stores, {bad} with an operand register rewritten before vmcnt(0)")
sys.exit(1 if bad else 0)
