"""Check that no instruction touches the destination registers of an inline-asm
global load before a wait covers it (the brick kernel's value and fill loads:
kle_sym_dev.hpp sym_ld9 / ld_x1, waited for by sym_wait9 / wait_x12 with an
explicit vmcnt that leaves younger loads in flight).  The compiler does not
know those registers are in flight: a copy or reuse of one before its data
lands reads or clobbers it (round 5: a two-items-ahead variant's registers were
moved -- wrong products).

  python tools/isa_inflight_check.py KERNEL.s [kernel-name-substring ...]

KERNEL.s from `hipcc --offload-arch=gfx950 --cuda-device-only -S`.  For each
asm load (a line between ;;#ASMSTART and ;;#ASMEND) it walks the control-flow
graph forward, counting vector-memory instructions issued after it (gfx9:
vmcnt counts loads and stores), until every path reaches an s_waitcnt whose
vmcnt(N) has N <= that count (the load is then complete); any instruction on
the way that names one of its destination VGPRs is reported.  Exit status 1
on a finding."""
import re
import sys

VM = re.compile(r"^\s*(global_|buffer_|flat_|scratch_)")
VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def vregs(text):
    out = set()
    for m in VREG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def kernels(lines):
    """(name, [lines]) of each kernel body in the .s"""
    cur, body = None, []
    for ln in lines:
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", ln)
        if m:
            cur, body = m.group(1), []
            continue
        if cur and ln.startswith(".Lfunc_end"):
            yield cur, body
            cur = None
        elif cur:
            body.append(ln)


def parse(body):
    """instructions [(text, in_asm)], label -> index, successors"""
    ins, labels, in_asm = [], {}, False
    for ln in body:
        s = ln.split(";")[0].strip() if not ln.strip().startswith(";;#ASM") else ln.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not s or s.startswith("."):
            if re.match(r"^\.LBB\S+:", s):
                labels[s[:-1]] = len(ins)
            continue
        if re.match(r"^\S+:$", s):
            labels[s[:-1]] = len(ins)
            continue
        ins.append((s, in_asm))
    return ins, labels


def succ(ins, labels, i, vcc=None):
    """successors of instruction i; vcc (True: nonzero, False: zero, None:
    unknown) prunes the vccz / vccnz branch that cannot be taken"""
    s = ins[i][0]
    op = s.split()[0]
    if op == "s_endpgm":
        return []
    if op == "s_branch":
        return [labels[s.split()[1]]]
    if op.startswith("s_cbranch"):
        t = labels[s.split()[1]]
        if op == "s_cbranch_vccz" and vcc is not None:
            return [i + 1] if vcc else [t]
        if op == "s_cbranch_vccnz" and vcc is not None:
            return [t] if vcc else [i + 1]
        return [t, i + 1]
    if op in ("s_setpc_b64", "s_swappc_b64"):
        return []
    return [i + 1] if i + 1 < len(ins) else []


def step_consts(s, consts, vcc):
    """the structurizer's flag idiom: s_mov_b64 s[a:b], -1 / 0 ... then
    s_and_b64 vcc, exec, s[a:b] and s_cbranch_vcc(n)z: known flags prune the
    paths that cannot run (exec is nonzero where an instruction runs)"""
    parts = s.replace(",", " ").split()
    op, dst = parts[0], parts[1] if len(parts) > 1 else ""
    consts = dict(consts)
    if op == "s_and_b64" and dst == "vcc" and len(parts) == 4 and parts[2] == "exec":
        v = consts.get(parts[3])
        vcc = None if v is None else v != 0
    elif dst in ("vcc", "vcc_lo", "vcc_hi") or (op.startswith("v_cmp") and "_e32" in op):
        vcc = None
    if op == "s_mov_b64" and len(parts) == 3 and parts[2] in ("-1", "0"):
        consts[dst] = int(parts[2])
    elif op.startswith("s_") and dst.startswith("s"):
        # (any other write of an SGPR pair or of one of its halves)
        for k in list(consts):
            lo, hi = map(int, k[2:-1].split(":"))
            m = re.match(r"^s\[(\d+):(\d+)\]$|^s(\d+)$", dst)
            if m:
                a = int(m.group(3) if m.group(3) else m.group(1))
                b2 = int(m.group(3) if m.group(3) else m.group(2))
                if a <= hi and b2 >= lo:
                    del consts[k]
    return tuple(sorted(consts.items())), vcc


def waitcnt(s):
    m = re.match(r"^s_waitcnt\b.*\bvmcnt\((\d+)\)", s)
    return int(m.group(1)) if m else None


def check(name, body):
    ins, labels = parse(body)
    bad = 0
    loads = [i for i, (s, a) in enumerate(ins) if a and s.startswith("global_load")]
    for li in loads:
        dst = vregs(ins[li][0].split(",")[0])
        # DFS over (instruction, vm ops since the load (capped), known flags)
        stack, seen = [(j, 0, (), None) for j in succ(ins, labels, li)], set()
        found = False
        while stack and not found:
            j, cnt, consts, vcc = stack.pop()
            if (j, cnt, consts, vcc) in seen or j >= len(ins):
                continue
            seen.add((j, cnt, consts, vcc))
            s, a = ins[j]
            n = waitcnt(s)
            if n is not None and n <= cnt:
                continue  # the load has landed on this path
            if vregs(s) & dst:
                print(f"{name[:60]}: load [{li}] '{ins[li][0]}' -> '{s}' [{j}] touches "
                      f"v{sorted(vregs(s) & dst)} with {cnt} vm ops after the load")
                bad += 1
                found = True  # (one report per load)
                continue
            if VM.match(s):
                cnt = min(cnt + 1, 64)
            consts, vcc = step_consts(s, consts, vcc)
            for k in succ(ins, labels, j, vcc):
                stack.append((k, cnt, consts, vcc))
    return bad, len(loads)


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    lines = open(path).read().split("\n")
    total = 0
    for name, body in kernels(lines):
        if subs and not any(x in name for x in subs):
            continue
        bad, n = check(name, body)
        print(f"{name[:90]}: {n} asm loads, {bad} findings")
        total += bad
    sys.exit(1 if total else 0)


if __name__ == "__main__":
    main()
