"""Per-kernel totals from a rocprofv3 SQLite result (run_results.db): the
--stats summary for runs whose output is the database.  Optional second
argument: count of timed steps to divide the totals by (µs a step)."""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    per = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    c = sqlite3.connect(db)
    rows = c.execute('select name, count(*), sum(duration) / 1000.0, avg(duration) / 1000.0 '
                     'from kernels group by name order by 3 desc limit 60').fetchall()
    tot = c.execute('select sum(duration) / 1000.0 from kernels').fetchone()[0]
    print('total us %.1f (per step %.1f)' % (tot, tot / per))
    print('%8s %12s %10s %10s  %s' % ('calls', 'total_us', 'avg_us', 'us/step', 'kernel'))
    for name, n, t, a in rows:
        print('%8d %12.1f %10.2f %10.2f  %s' % (n, t, a, t / per, name[:120]))


if __name__ == '__main__':
    main()
