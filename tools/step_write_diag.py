"""tools/step_write_diag.sh helpers: `build` compiles the store-masked
diagnostic libraries (CPU, here); `report` prints step_fan_kernel's mean
WRITE_SIZE per dispatch for each mask from gpurun_out/stw_<mask>/."""
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
MASKS = (0, 1, 2, 4, 8, 16)
NAMES = {0: 'all stores', 1: '-reward', 2: '-reward_mod', 4: '-done', 8: '-obs', 16: '-refill'}


def build():
    from aido1_amd import _lib
    for m in MASKS:
        _lib.build(force=True, path=os.path.join(_lib.PKG_DIR, 'libdtsim_diag_st%d.so' % m),
                   defines=['DTSIM_DIAG_SKIP_STORES=%d' % m])
        print('built mask', m)


def report():
    base = None
    for m in MASKS:
        vals = []
        for f in glob.glob('gpurun_out/stw_%d/**/*counter_collection.csv' % m, recursive=True):
            for r in csv.DictReader(open(f)):
                if 'step_fan_kernel' in r['Kernel_Name'] and r['Counter_Name'] == 'WRITE_SIZE':
                    vals.append(float(r['Counter_Value']))
        if not vals:
            print(m, 'no data')
            continue
        kib = sum(vals) / len(vals)
        base = kib if m == 0 else base
        print('%-12s %8.1f KiB per launch  (%+.1f)' % (NAMES[m], kib, kib - base))


if __name__ == '__main__':
    {'build': build, 'report': report}[sys.argv[1]]()
