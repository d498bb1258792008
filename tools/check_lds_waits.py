"""Static check of a gfx950 .s file: no instruction may read a VGPR/AGPR that is the destination of
an LDS read (ds_read*) still in flight, i.e. not yet retired by an s_waitcnt lgkmcnt(N), and no
instruction may overwrite one (the late LDS return would clobber it).

Kernels that issue LDS reads through inline asm (csrc/kernels/softmax_grad_dw.hip) manage lgkmcnt
themselves; if the register allocator ever copied an asm read's destination before the counted wait,
the copy would read stale data with no fault. This runs a dataflow over each kernel's basic blocks
(pending-read queues merged per predecessor, aligned from the newest entry since a wait keeps the
newest N) and reports such accesses. Usage: python tools/check_lds_waits.py file.s [kernel-substring]
"""
import re
import sys

QMAX = 16
REG = re.compile(r"\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1):
            out |= {(m.group(1), r) for r in range(int(m.group(2)), int(m.group(3)) + 1)}
        else:
            out.add((m.group(4), int(m.group(5))))
    return out


def parse(lines):
    """-> list of (no, op, rest, raw) instructions and label -> index."""
    ins, labels = [], {}
    for no, raw in lines:
        ln = raw.split(";")[0].strip()
        if not ln:
            continue
        if ln.endswith(":"):
            labels[ln[:-1]] = len(ins)
            continue
        if ln.startswith("."):
            continue
        op, _, rest = ln.partition(" ")
        ins.append((no, op, rest.strip(), raw.strip()))
    return ins, labels


def merge(qs):
    """Pending queues aligned from the newest entry (a wait keeps the newest N)."""
    n = max(len(q) for q in qs)
    out = []
    for k in range(n, 0, -1):
        out.append(frozenset().union(*[q[-k] for q in qs if len(q) >= k]))
    return tuple(out)


def step(q, op, rest):
    """-> (new queue, registers this instruction touches that are still in flight)."""
    if op == "s_waitcnt":
        m = re.search(r"lgkmcnt\((\d+)\)", rest)
        if m:
            keep = int(m.group(1))
            q = q[len(q) - keep:] if keep else ()
        return q, set()
    operands = [o.strip() for o in rest.split(",")]
    is_read = op.startswith("ds_read") or op.startswith("ds_load")
    if is_read:
        srcs, dst = regs(",".join(operands[1:])), regs(operands[0])
    elif op.startswith("ds_") or "store" in op:
        srcs, dst = regs(rest), set()
    else:
        srcs, dst = regs(",".join(operands[1:])), (regs(operands[0]) if operands else set())
    live = set().union(*q) if q else set()
    hit = (srcs | (set() if is_read else dst)) & live
    if is_read:
        q = q + (frozenset(dst),)
    elif op.startswith("ds_") or op.startswith("s_load") or op.startswith("s_buffer_load"):
        q = q + (frozenset(),)
    if len(q) > QMAX:  # a wait keeps at most 15: entries older than that retire together
        q = (q[0] | q[1],) + q[2:]
    return q, hit


def check(lines, name):
    ins, labels = parse(lines)
    # basic blocks: leaders are label targets and instructions after a branch
    leaders = sorted({0} | set(labels.values()) |
                     {i + 1 for i, (_, op, _, _) in enumerate(ins) if op.startswith("s_branch") or op.startswith("s_cbranch")})
    leaders = [l for l in leaders if l < len(ins)]
    bounds = {l: (leaders[k + 1] if k + 1 < len(leaders) else len(ins)) for k, l in enumerate(leaders)}
    entry = {0: ()}
    bad = {}
    work = [0]
    visits = 0
    while work and visits < 20000:
        visits += 1
        b = work.pop()
        q = entry[b]
        for i in range(b, bounds[b]):
            no, op, rest, raw = ins[i]
            q, hit = step(q, op, rest)
            if hit:
                bad[no] = (raw, sorted(hit)[:4])
        last = ins[bounds[b] - 1][1]
        succ = []
        if last.startswith("s_branch"):
            succ = [labels.get(ins[bounds[b] - 1][2])]
        elif last.startswith("s_cbranch"):
            succ = [labels.get(ins[bounds[b] - 1][2]), bounds[b]]
        elif last != "s_endpgm":
            succ = [bounds[b]]
        for sb in succ:
            if sb is None or sb >= len(ins):
                continue
            new = merge([entry[sb], q]) if sb in entry else q
            if entry.get(sb) != new:
                entry[sb] = new
                work.append(sb)
    if work:  # did not converge: report it rather than a clean result
        bad[0] = ("dataflow did not converge", [])
    return [(no, raw, hit) for no, (raw, hit) in sorted(bad.items())]


def kernels(path, sub):
    cur, body = None, []
    for no, line in enumerate(open(path), 1):
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m:
            if cur and sub in cur:
                yield cur, body
            cur, body = m.group(1), []
        elif cur is not None:
            body.append((no, line))
            if "s_endpgm" in line:
                if sub in cur:
                    yield cur, body
                cur, body = None, []


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    total = 0
    for name, body in kernels(path, sub):
        bad = check(body, name)
        total += len(bad)
        print(f"{name[:90]}: {len(bad)} reads of in-flight LDS destinations")
        for no, ins, hit in bad[:10]:
            print(f"  line {no}: {ins}   {hit}")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
