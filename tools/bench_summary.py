"""Print the headline and sub-record figures of a bench.py JSON line."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('headline %.4gM  ms/step %.4f  frac %.4f  kernel %.4f ms  parity ok %s' % (
    d['value'] / 1e6, d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_kernel_ms'],
    (d.get('parity') or {}).get('ok')))
for k in ('config2', 'config4', 'config4_fp16', 'config5', 'config5_fp16'):
    r = d.get(k)
    if not r:
        continue
    rf = r['roofline']
    par = r.get('parity') or {}
    extra = ''
    if 'max_abs_err_vs_f64' in par:
        extra = ' |da|f64 %.3g (%d envs)' % (par['max_abs_err_vs_f64'], par['envs_checked_f64'])
    if r.get('phases_ms'):
        extra += ' actor %.3f update %.3f ms' % (r['phases_ms']['actor'], r['phases_ms']['update'] or 0)
    print('%-13s %.4gM ms/step %.3f  %s %.4g %s frac %.3f ok %s%s' % (
        k, r['value'] / 1e6, r['ms_per_step'], rf['bound'], rf['achieved'], rf['unit'],
        rf['frac'], par.get('ok'), extra))
