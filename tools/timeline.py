"""Print the kernel timeline of one bench step from a rocprofv3 sqlite db (start/end relative, us)."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
step = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rows = list(c.execute("select s.kernel_name, d.start, d.end, d.stream_id from rocpd_kernel_dispatch d "
                      "join rocpd_info_kernel_symbol s on d.kernel_id=s.id order by d.start"))
# steps begin at each k_pyramid_level<true>
starts = [i for i, r in enumerate(rows) if "k_pyramid_levelILb1" in r[0]]
i0, i1 = starts[step], starts[step + 1] if step + 1 < len(starts) else len(rows)
t0 = rows[i0][1]
for name, st, en, sid in rows[i0:i1]:
    short = name.split("(")[0].replace("_ZN12_GLOBAL__N_1", "")[:48]
    print(f"{short:50s} stream {sid:3d}  {(st - t0) / 1e3:8.1f} -> {(en - t0) / 1e3:8.1f}  ({(en - st) / 1e3:6.1f})")
print("step span", (rows[i1 - 1][2] - t0) / 1e3)
