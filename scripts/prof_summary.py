"""Per-kernel launch counts and average durations from rocprofv3 result databases (the rocpd
SQLite output of `rocprofv3 --kernel-trace`):  python scripts/prof_summary.py <db> [<db> ...] [--grep s]"""
import sqlite3
import sys


def summary(db, pat=None):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), avg(end - start) / 1000.0, sum(end - start) / 1000.0 "
                     "from kernels group by name order by 4 desc").fetchall()
    return [r for r in rows if not pat or pat in r[0]]


if __name__ == "__main__":
    args = sys.argv[1:]
    pat = None
    if "--grep" in args:
        i = args.index("--grep")
        pat = args[i + 1]
        del args[i:i + 2]
    for db in args:
        print(db)
        for name, n, avg, tot in summary(db, pat):
            short = name.split("(")[0].replace("void ", "")
            print(f"  {short[:56]:56s} {n:5d} x {avg:10.1f} us  (total {tot:10.1f})")
