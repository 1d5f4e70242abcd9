"""tools/render_phase_valu.sh helpers: `build` the phase-stop diagnostic
libraries (CPU, here); `report` the per-dispatch instruction counts of
render_kernel per build and their differences (the phases' shares)."""
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
STOPS = ('1', '2', '3', '4', 'full')
NAMES = {'1': 'spans + projection', '2': '+ fix-up, markings', '3': '+ uniformity',
         '4': '+ Canny (Sobel, NMS, hysteresis)', 'full': '+ outputs'}


def build():
    from aido1_amd import _lib
    for k in STOPS:
        d = [] if k == 'full' else ['DTSIM_RENDER_STOP_AT=%s' % k]
        _lib.build(force=True, path=os.path.join(_lib.PKG_DIR, 'libdtsim_rstop_%s.so' % k),
                   defines=d)
        print('built', k)


def report():
    prev = None
    for k in STOPS:
        acc = {}
        for f in glob.glob('gpurun_out/rstop_%s/**/*counter_collection.csv' % k, recursive=True):
            for r in csv.DictReader(open(f)):
                if 'render_kernel' in r['Kernel_Name']:
                    acc.setdefault(r['Counter_Name'], []).append(float(r['Counter_Value']))
        if not acc:
            print(k, 'no data')
            continue
        m = {c: sum(v) / len(v) for c, v in acc.items()}
        waves = m.get('SQ_WAVES', 1.0)
        line = '%-34s' % NAMES[k]
        for c in ('SQ_INSTS_VALU', 'SQ_INSTS_LDS', 'SQ_INSTS_SALU'):
            per = m.get(c, 0.0) / waves
            d = per - (prev[c] if prev else 0.0)
            line += '  %s %7.0f/wave (+%6.0f)' % (c[9:], per, d)
        print(line)
        prev = {c: m.get(c, 0.0) / waves for c in m}


if __name__ == '__main__':
    {'build': build, 'report': report}[sys.argv[1]]()
