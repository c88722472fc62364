"""Per-kernel time summary from a rocprofv3 SQLite output (rocpd *_results.db): calls, total,
mean, min, max (us) per kernel, sorted by total.  Usage: python tools/rocpd_stats.py DB [--tsv OUT]"""
import argparse
import sqlite3
import statistics


def stats(db: str) -> list[tuple]:
    c = sqlite3.connect(db)
    names = {r[0]: r[1] for r in c.execute("select id, coalesce(display_name, kernel_name) from rocpd_info_kernel_symbol")}
    per: dict[str, list[float]] = {}
    for kid, s, e in c.execute("select kernel_id, start, end from rocpd_kernel_dispatch"):
        per.setdefault(names.get(kid, str(kid)), []).append((e - s) / 1e3)
    rows = [(k, len(v), sum(v), statistics.mean(v), min(v), max(v)) for k, v in per.items()]
    return sorted(rows, key=lambda r: -r[2])


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--tsv")
    a = ap.parse_args()
    rows = stats(a.db)
    lines = ["kernel\tcalls\ttotal_us\tmean_us\tmin_us\tmax_us"] + \
            [f"{k[:110]}\t{n}\t{t:.1f}\t{m:.1f}\t{lo:.1f}\t{hi:.1f}" for k, n, t, m, lo, hi in rows]
    print("\n".join(lines))
    if a.tsv:
        open(a.tsv, "w").write("\n".join(lines) + "\n")
