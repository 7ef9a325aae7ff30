"""Summarise a rocprofv3 sqlite results file: per-kernel count, average and total time."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
q = ("select s.kernel_name, count(*), avg(d.end-d.start)/1000.0, sum(d.end-d.start)/1e6 "
     "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id=s.id "
     "group by s.kernel_name order by 4 desc")
print(f"{'kernel':70s} {'calls':>7s} {'avg_us':>10s} {'total_ms':>10s}")
for name, n, avg, tot in c.execute(q):
    print(f"{name[:70]:70s} {n:7d} {avg:10.2f} {tot:10.3f}")
