"""Summarise a tools/profile_round.sh run: copy the kernel-trace stats into
profiles/<round>_<config>_kernel_stats.csv and turn the PMC passes into
profiles/pmc_traffic.json (per-launch HBM bytes of the dominant kernels).

Corrections (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE reports
half the bytes of wide coalesced streaming reads, so it is doubled; WRITE_SIZE
is exact for 16-B-per-lane stores.  Both are in KiB per dispatch."""
import csv
import glob
import json
import os
import shutil
import sys

ROUND = sys.argv[1] if len(sys.argv) > 1 else 'r01'
OUT = 'gpurun_out'
KERNELS = {'lane': [('step_pair_kernel', ['step_pair_kernel']), ('step_kernel', ['step_kernel'])],
           'render': [('render_kernel', ['render_kernel'])]}


def per_dispatch(path, needle):
    vals = {}
    for row in csv.DictReader(open(path)):
        name = row.get('Kernel_Name', '')
        if needle + '(' not in name and not name.endswith(needle):
            continue
        key = row.get('Dispatch_Id') or row.get('Correlation_Id')
        vals[key] = vals.get(key, 0.0) + float(row['Counter_Value'])
    return sum(vals.values()) / len(vals) if vals else None


def main():
    for d in sorted(glob.glob(os.path.join(OUT, 'trace_*'))):
        cfg = d.split('trace_', 1)[1]
        for f in glob.glob(os.path.join(d, '**', '*kernel_stats.csv'), recursive=True):
            shutil.copy(f, 'profiles/%s_%s_kernel_stats.csv' % (ROUND, cfg))
            print('copied', f)
    out = {}
    if os.path.exists('profiles/pmc_traffic.json'):   # keep kernels this run did not profile
        with open('profiles/pmc_traffic.json') as f:
            out = json.load(f)
    for cfg, label, names in [(c, l, n) for c, ks in KERNELS.items() for l, n in ks]:
        fetch = write = 0.0
        ok = True
        for ctr in ('FETCH_SIZE', 'WRITE_SIZE'):
            files = glob.glob(os.path.join(OUT, 'pmc_%s_%s' % (cfg, ctr), '**',
                                           '*counter_collection.csv'), recursive=True)
            if not files:
                ok = False
                continue
            for n in names:
                v = per_dispatch(files[0], n)
                if v is None:
                    ok = False
                    continue
                if ctr == 'FETCH_SIZE':
                    fetch += v
                else:
                    write += v
        if ok:
            out[label] = {'fetch_kib_raw': fetch, 'write_kib': write,
                          'hbm_bytes_per_launch': (2 * fetch + write) * 1024.0,
                          'note': 'FETCH_SIZE doubled (gfx950 half-count of wide reads); '
                                  'per dispatch, averaged; summed over %s' % '+'.join(names)}
    if out:
        with open('profiles/pmc_traffic.json', 'w') as f:
            json.dump(out, f, indent=1)
        print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
