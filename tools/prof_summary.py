"""Summarise a rocprofv3 rocpd database (kernel dispatch stats) into CSV on stdout."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else "name"
q = f"""select {name}, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start)
        from kernels group by {name} order by sum(end-start) desc"""
rows = list(c.execute(q))
tot = sum(r[2] for r in rows) or 1
print("kernel,calls,total_ns,avg_ns,min_ns,max_ns,pct")
for n, k, s, a, mn, mx in rows:
    print(f'"{n[:120]}",{k},{s},{a:.0f},{mn},{mx},{100.0 * s / tot:.2f}')
