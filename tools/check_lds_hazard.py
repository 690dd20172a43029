"""Static check on a disassembled code object: no instruction reads a ds_read's destination VGPRs
before the read has completed.

    llvm-objdump -d lib.co > lib.dis
    python tools/check_lds_hazard.py lib.dis [kernel-substring]

The kernels issue their LDS fragment reads as inline asm and tie each one to a counted
`s_waitcnt lgkmcnt(N)` (siren_fwdreg.hip freg_read / freg_lgkm, siren_gemm.hip ring_chain). The
compiler takes an asm output as defined at the asm, so if register allocation ever moves one
(a v_mov at a control-flow merge) before its wait, the copy reads stale bytes: round 3 saw exactly
that (a runtime branch at a block boundary, one wave's block wrong in a few runs out of 100).
For every ds_read, every control-flow path from it is followed until a wait guarantees it has
landed — lgkmcnt(N) with at least N younger LDS operations on that path (LDS completes in order;
an outstanding scalar load makes only lgkmcnt(0) count) — and any instruction reading one of its
destination registers before that is reported. Exit status 1 if any is found."""
import re
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
path = args[0]
filt = args[1] if len(args) > 1 else "fused_fwd_reg_kernel"

kernels = {}
cur = None
for line in open(path).read().split("\n"):
    m = re.match(r"^([0-9a-f]+) <(\S+)>:", line)
    if m:
        cur = m.group(2) if filt in m.group(2) else None
        if cur:
            kernels[cur] = (int(m.group(1), 16), [])
        continue
    if not cur or not line.strip():
        continue
    m = re.match(r"^\s*(\S.*?)\s*//\s*([0-9A-Fa-f]+):[^<]*(?:<(\S+?)(?:\+0x([0-9a-f]+))?>)?", line)
    if not m:
        continue
    ins, addr = m.group(1).strip(), int(m.group(2), 16)
    tgt = None
    if m.group(3) and ins.startswith(("s_branch", "s_cbranch")):
        base = kernels[cur][0] if m.group(3) == cur else None
        if base is not None:
            tgt = base + int(m.group(4) or "0", 16)
    kernels[cur][1].append((addr, ins, tgt))


def vregs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def ops(ins):
    t = ins.split(None, 1)
    return [x.strip() for x in t[1].split(",")] if len(t) > 1 else []


def reads(ins):
    """VGPRs an instruction reads (every operand but the destination; for stores every operand)."""
    op = ins.split()[0]
    o = ops(ins)
    if not o or op.startswith("s_"):
        return set()
    srcs = o if op.startswith(("buffer_store", "global_store", "scratch_store", "ds_write")) else o[1:]
    r = set()
    for x in srcs:
        r |= vregs(x.split()[0] if x else x)
    return r


def is_lds(ins):
    return ins.startswith("ds_")


def is_smem(ins):
    return ins.startswith(("s_load", "s_buffer_load"))


bad = nreads = 0
for name, (base, body) in kernels.items():
    index = {addr: i for i, (addr, _, _) in enumerate(body)}

    def succ(i):
        _, ins, tgt = body[i]
        if ins.startswith("s_endpgm"):
            return []
        out = []
        if tgt is not None and tgt in index:
            out.append(index[tgt])
        if not ins.startswith("s_branch") and i + 1 < len(body):
            out.append(i + 1)
        return out

    for i, (_, ins, _) in enumerate(body):
        if not ins.startswith("ds_read"):
            continue
        nreads += 1
        dst = vregs(ops(ins)[0])
        # state: (instruction, younger LDS ops, scalar load outstanding)
        seen, stack, hit = set(), [(k, 0, False) for k in succ(i)], None
        while stack and hit is None:
            j, young, sm = stack.pop()
            if (j, young, sm) in seen:
                continue
            seen.add((j, young, sm))
            w = body[j][1]
            m = re.match(r"s_waitcnt .*lgkmcnt\((\d+)\)", w)
            if m and (int(m.group(1)) == 0 or (not sm and young >= int(m.group(1)))):
                continue
            if reads(w) & dst:
                hit = j
                break
            if is_lds(w):
                young = min(young + 1, 32)
            if is_smem(w):
                sm = True
            stack.extend((k, young, sm) for k in succ(j))
        if hit is not None:
            bad += 1
            if bad <= 20:
                print(f"{name[:60]} @{body[i][0]:x}: {ins}  <- read @{body[hit][0]:x}: {body[hit][1]}")
print(f"{len(kernels)} kernels, {nreads} LDS reads, {bad} with a destination read before the read completed")
sys.exit(1 if bad else 0)
