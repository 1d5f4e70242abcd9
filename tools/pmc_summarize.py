"""Summarise a tools/profile_round.sh run: copy the kernel-trace stats into
profiles/<round>_<config>_kernel_stats.csv and turn the PMC passes into
profiles/pmc_traffic.json (per-launch HBM bytes and fp64 instruction counts of
the dominant kernels).

FETCH_SIZE correction (MI355X_MICROARCH.md, HBM section): on gfx950
FETCH_SIZE reports half the bytes of a WIDE coalesced streaming read (16 B per
lane, global_load_dwordx4 / buffer_load ... lds).  Only kernels whose reads are
of that kind get it doubled (WIDE_READS below); the step and render kernels
read 4-8 B per lane (f64 state, u32 slot words, LDS-staged map), where the
note does not apply, so their FETCH_SIZE is taken as is.  Both readings are
recorded.  WRITE_SIZE is exact for 16-B-per-lane stores.  Both are KiB per
dispatch."""
import csv
import glob
import json
import os
import shutil
import sys

if len(sys.argv) < 2:   # it writes profiles/<round>_*: no default round to overwrite
    sys.exit('usage: python tools/pmc_summarize.py <round, e.g. r03>')
ROUND = sys.argv[1]
OUT = 'gpurun_out'
# label -> (bench config whose PMC passes hold it, kernel-name needles)
KERNELS = {'step_fan_kernel': ('lane', ['step_fan_kernel']),
           'step_kernel': ('lane', ['step_kernel']),
           'render_kernel': ('render', ['render_kernel'])}
WIDE_READS = set()      # kernels whose reads are 16-B-per-lane streams
FP64 = ('SQ_INSTS_VALU_ADD_F64', 'SQ_INSTS_VALU_MUL_F64', 'SQ_INSTS_VALU_FMA_F64',
        'SQ_INSTS_VALU_TRANS_F64')


def per_dispatch(path, needle, counter=None):
    vals = {}
    for row in csv.DictReader(open(path)):
        name = row.get('Kernel_Name', '')
        if needle + '(' not in name and needle + '<' not in name and not name.endswith(needle):
            continue
        if counter and row.get('Counter_Name') != counter:
            continue
        key = row.get('Dispatch_Id') or row.get('Correlation_Id')
        vals[key] = vals.get(key, 0.0) + float(row['Counter_Value'])
    return sum(vals.values()) / len(vals) if vals else None


def pmc_files(cfg, tag):
    return glob.glob(os.path.join(OUT, 'pmc_%s_%s' % (cfg, tag), '**', '*counter_collection.csv'),
                     recursive=True)


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
    for label, (cfg, names) in KERNELS.items():
        rec = {}
        for ctr in ('FETCH_SIZE', 'WRITE_SIZE'):
            files = pmc_files(cfg, ctr)
            vals = [per_dispatch(files[0], n) for n in names] if files else [None]
            if any(v is None for v in vals):
                rec = None
                break
            rec[ctr] = sum(vals)
        if rec:
            fetch, write = rec['FETCH_SIZE'], rec['WRITE_SIZE']
            wide = label in WIDE_READS
            r = {'round': ROUND, 'fetch_kib_raw': fetch, 'write_kib': write,
                 'hbm_bytes_per_launch': ((2 if wide else 1) * fetch + write) * 1024.0,
                 'hbm_bytes_per_launch_fetch_doubled': (2 * fetch + write) * 1024.0,
                 'hbm_bytes_per_launch_fetch_raw': (fetch + write) * 1024.0,
                 'fetch_doubled': wide,
                 'note': 'per dispatch, averaged; FETCH_SIZE %s (gfx950 half-count applies '
                         'to 16-B/lane streaming reads only)' % ('doubled' if wide else 'raw')}
            old = out.get(label, {})
            if label.startswith('step_'):
                r['decisions_per_launch'] = int(os.environ.get('PMC_DECISIONS', '20'))
            out[label] = {**{k: v for k, v in old.items() if k.startswith('fp64')}, **r}
        files = pmc_files(cfg, 'FP64')
        if files:
            cnt = {c: per_dispatch(files[0], names[0], c) for c in FP64}
            if all(v is not None for v in cnt.values()):
                # wave-instructions -> lane flops (64 lanes; an FMA is 2 flops)
                flops = 64.0 * (cnt['SQ_INSTS_VALU_ADD_F64'] + cnt['SQ_INSTS_VALU_MUL_F64'] +
                                cnt['SQ_INSTS_VALU_TRANS_F64'] + 2 * cnt['SQ_INSTS_VALU_FMA_F64'])
                out.setdefault(label, {})
                out[label]['fp64_insts_per_launch'] = cnt
                out[label]['fp64_flops_per_launch'] = flops
    if out:
        with open('profiles/pmc_traffic.json', 'w') as f:
            json.dump(out, f, indent=1)
        print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
