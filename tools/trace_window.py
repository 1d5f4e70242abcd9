"""One window of a rocprofv3 kernel trace as a timeline: every kernel between
the n-th and (n+1)-th start of a marker kernel, with its start offset, duration,
queue and the idle gaps of the device.
usage: python tools/trace_window.py TRACE.csv MARKER_SUBSTRING [N]"""
import csv
import sys


def main():
    path, marker = sys.argv[1], sys.argv[2]
    nth = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'],
                         r['Queue_Id'], int(r['Grid_Size_X']) // max(1, int(r['Workgroup_Size_X']))))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if marker in r[2]]
    a, b = starts[nth], starts[nth + 1]
    t0 = rows[a][0]
    busy_end = t0
    idle = 0
    for s, e, name, q, wgs in rows[a:b]:
        gap = max(0, s - busy_end)
        idle += gap
        busy_end = max(busy_end, e)
        print('%8.1f %7.1f  gap %6.1f  q%s wg %6d  %s' % ((s - t0) / 1e3, (e - s) / 1e3, gap / 1e3, q,
                                                        wgs, name[:90]))
    print('window %.1f us, %d kernels, device idle %.1f us'
          % ((rows[b][0] - t0) / 1e3, b - a, idle / 1e3))


if __name__ == '__main__':
    main()
