"""Per-kernel stats (calls, total/avg us, share) from a rocprofv3 rocpd SQLite database.
    python tools/prof_db_stats.py <results.db> [top]"""
import sqlite3
import sys


def main(path, top=25):
    con = sqlite3.connect(path)
    q = """select s.display_name, count(*), sum(d.end - d.start), avg(d.end - d.start)
           from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
           group by s.display_name order by sum(d.end - d.start) desc"""
    rows = con.execute(q).fetchall()
    tot = sum(r[2] for r in rows)
    print(f"{'kernel':70s} {'calls':>6s} {'total_us':>10s} {'avg_us':>9s} {'share':>6s}")
    for name, n, s, a in rows[:top]:
        print(f"{name[:70]:70s} {n:6d} {s / 1e3:10.1f} {a / 1e3:9.2f} {100 * s / tot:5.1f}%")
    print(f"total kernel time {tot / 1e3:.1f} us over {sum(r[1] for r in rows)} dispatches")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25)
