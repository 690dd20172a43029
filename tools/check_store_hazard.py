"""Static check of the store-hazard rule (siren_common.h) on a disassembled code object:
    llvm-objdump -d lib.co > lib.dis
    python tools/check_store_hazard.py lib.dis [kernel-substring] [--all-operands]
For every buffer / scratch / global store in the matching kernels, follow every control-flow path
from the store (branch targets included) and report an instruction that writes one of the store's
data VGPRs (--all-operands: also the address VGPR and descriptor SGPRs of buffer stores) before an
s_waitcnt vmcnt(N) with at least N vector-memory operations issued after the store on that path
(vmcnt counts in issue order: then the store has completed, the only thing that guarantees it has
read them) — or the program end (the original, conservative rule).
Exit status 1 if any store violates the rule.

--window=N: the measured rule instead (tools/probe_store_hazard.hip): on gfx950 a
store of more than 8 bytes reads its data VGPRs during the two wait states after its issue (a
VALU write of them with no wait state in between corrupts lanes 8-15 of each 16-lane group, with
one — one instruction or s_nop 0 — lanes 12-15; with two — s_nop 1, or two instructions — none, in
2.7e9 stores, with or without LDS-DMA or other stores in flight). A violation is then a write of a
data VGPR with fewer than N wait states after the store on some path (s_nop k = k + 1 wait states,
any other instruction 1; N = 2 is the measured requirement), unless a vmcnt wait covers the store."""
import re
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
path = args[0]
filt = args[1] if len(args) > 1 else "fused_fwd_reg_kernel"
ALL = "--all-operands" in sys.argv
WINDOW = next((int(a.split("=", 1)[1]) for a in sys.argv if a.startswith("--window=")), None)

kernels = {}  # name -> (base address, [(addr, ins, target addr or None)])
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
        return {("v", r) for r in range(int(m.group(1)), int(m.group(2)) + 1)}
    m = re.match(r"v(\d+)$", tok)
    return {("v", int(m.group(1)))} if m else set()


def sregs(tok):
    m = re.match(r"s\[(\d+):(\d+)\]", tok)
    if m:
        return {("s", r) for r in range(int(m.group(1)), int(m.group(2)) + 1)}
    m = re.match(r"s(\d+)$", tok)
    return {("s", int(m.group(1)))} if m else set()


def ops(ins):
    t = ins.split(None, 1)
    return [x.strip() for x in t[1].split(",")] if len(t) > 1 else []


def store_regs(ins):
    o = ops(ins)
    if ins.startswith("buffer_store"):
        r = vregs(o[0])
        if ALL:
            r |= vregs(o[1]) | (sregs(o[2]) if len(o) > 2 else set())
        return r
    return vregs(o[1]) if len(o) > 1 else set()  # scratch_store / global_store ADDR, DATA


def writes(ins):
    op = ins.split()[0]
    if op.startswith(("buffer_store", "global_store", "scratch_store", "ds_write")) or "_lds" in op:
        return set()
    o = ops(ins)
    if not o:
        return set()
    if op.startswith("s_"):
        if op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_cbranch", "s_branch", "s_setprio", "s_sleep",
                          "s_endpgm", "s_dcache", "s_sethalt", "s_trap")):
            return set()
        return sregs(o[0])
    return vregs(o[0]) | sregs(o[0])


bad = nstores = 0
for name, (base, body) in kernels.items():
    index = {addr: i for i, (addr, _, _) in enumerate(body)}

    def succ(i):
        addr, ins, tgt = body[i]
        if ins.startswith("s_endpgm"):
            return []
        out = []
        if tgt is not None and tgt in index:
            out.append(index[tgt])
        if not ins.startswith("s_branch") and i + 1 < len(body):
            out.append(i + 1)
        return out

    for i, (_, ins, _) in enumerate(body):
        if not ins.startswith(("buffer_store", "scratch_store", "global_store")):
            continue
        if WINDOW is not None and not re.match(r"\S+_store_dwordx[34]\b", ins):
            continue  # the measured window: stores of more than 8 bytes (probe_store_hazard.hip)
        nstores += 1
        data = store_regs(ins)
        # DFS over (instruction, vector-memory operations issued after the store on this path): a
        # wait vmcnt(N) with at least N of them younger means the store has completed (vmcnt counts
        # in issue order)
        seen, stack, hit = set(), [(k, 0, 0) for k in succ(i)], None
        while stack and hit is None:
            j, young, dist = stack.pop()
            if (j, young, dist) in seen:
                continue
            seen.add((j, young, dist))
            w = body[j][1]
            if WINDOW is not None:
                m = re.match(r"s_waitcnt .*vmcnt\((\d+)\)", w)
                # dist = wait states issued since the store before instruction j
                if dist >= WINDOW or (m and young >= int(m.group(1))):
                    continue
                if writes(w) & data:
                    hit = j
                    break
                if w.startswith(("buffer_", "global_", "scratch_")):
                    young = min(young + 1, 64)
                mn = re.match(r"s_nop\s+(?:0x)?([0-9a-f]+)", w)
                ws = int(mn.group(1), 16 if "0x" in w else 10) + 1 if mn else 1
                stack.extend((k, young, dist + ws) for k in succ(j))
                continue
            m = re.match(r"s_waitcnt .*vmcnt\((\d+)\)", w)
            if m and young >= int(m.group(1)):
                continue
            if writes(w) & data:
                hit = j
                break
            if w.startswith(("buffer_", "global_", "scratch_")):
                young = min(young + 1, 64)
            stack.extend((k, young, 0) for k in succ(j))
        if hit is not None:
            bad += 1
            print(f"{name[:60]} @{body[i][0]:x}: {ins}  <- written @{body[hit][0]:x}: {body[hit][1]}")
print(f"{len(kernels)} kernels, {nstores} stores, {bad} with a {'store operand' if ALL else 'data'} register "
      + (f"rewritten with fewer than {WINDOW} wait states after the store" if WINDOW is not None
         else "rewritten before the store completed (vmcnt)") + " on some path")
sys.exit(1 if bad else 0)
