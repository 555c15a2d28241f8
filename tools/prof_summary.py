"""Per-kernel summary of a rocprofv3 results database (kernel-trace): total / count /
average duration, sorted by total. Usage: prof_summary.py <run_results.db> [top]"""
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    rows = db.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                      "from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows)
    print("total_ms,pct,calls,avg_us,min_us,max_us,kernel")
    for name, n, s, a, lo, hi in rows[:top]:
        print(f"{s / 1e6:.3f},{100 * s / tot:.1f},{n},{a / 1e3:.1f},{lo / 1e3:.1f},{hi / 1e3:.1f},\"{name[:140]}\"")
    print(f"{tot / 1e6:.3f},100.0,{sum(r[1] for r in rows)},,,,TOTAL")


if __name__ == "__main__":
    main()
