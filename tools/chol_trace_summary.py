"""Summarise the MFTRACE stamps of tools/ba_trace.py (ORBGPU_BA_TRACE=1, k_ba_chol_mf2): per forward
step the diagonal wave's wait / compute and the tile waves' update window; the backward phase; the
diagonal factor phases.  Cycles are s_memtime ticks (shader clock)."""
import re
import sys

L = open(sys.argv[1]).read().split("\n")
steps, diag = {}, []
for l in L:
    m = re.match(r"MFTRACE k=(\d+) w=(\d+) (-?\d+) (-?\d+) (-?\d+) (-?\d+)", l)
    if m:
        steps[(int(m[1]), int(m[2]))] = tuple(int(x) for x in m.groups()[2:])
    m = re.match(r"MFTRACE diag k=(\d+) factor (-?\d+) linv (-?\d+) y (-?\d+)", l)
    if m:
        diag.append(tuple(int(x) for x in m.groups()[1:]))
W = max(w for _, w in steps)
back = [int(m[1]) for m in (re.match(r"MFTRACE back k=\d+ (-?\d+)", l) for l in L) if m]
end = [int(m[1]) for m in (re.match(r"MFTRACE end (-?\d+)", l) for l in L) if m]
nt = max(k for k, _ in steps) + 1
fwd_end = steps[(nt - 2, W)][3] if (nt - 2, W) in steps else -1
print(f"forward {fwd_end} cycles ({nt - 1} steps, {fwd_end / max(1, nt - 1):.0f}/step), backward "
      f"{end[0] - max(back) if end and back else -1}, total {end[0] if end else -1}")
for k in range(nt - 1):
    d = steps[(k, W)]
    print(f"  k={k:2d} diag wait {d[2] - d[1]:6d} compute {d[3] - d[2]:6d}   factor {diag[k][0]:6d}")
