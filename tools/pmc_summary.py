"""Summarise rocprofv3 PMC passes of the dominant kernel into profiles/<name>.json.

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reads half the bytes of a wide coalesced stream, so
traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.

usage: python tools/pmc_summary.py <pmc_dir> <out.json> <kernel-substring> [config-json]
(the config records the engine-source hash; bench.py attaches the traffic only on a match)
"""
import csv, glob, json, os, sys, collections

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (source_hash: the summary is valid for these engine sources only)

pmc_dir, out, kname = sys.argv[1:4]
config = json.loads(sys.argv[4]) if len(sys.argv) > 4 else {}
config['src_hash'] = bench.source_hash()
vals = collections.defaultdict(list)
durs = []
for f in sorted(glob.glob(f'{pmc_dir}/p*/pmc_counter_collection.csv')):
    for row in csv.DictReader(open(f)):
        if kname not in row['Kernel_Name']:
            continue
        vals[row['Counter_Name']].append(float(row['Counter_Value']))
        durs.append(int(row['End_Timestamp']) - int(row['Start_Timestamp']))
mean = {k: sum(v) / len(v) for k, v in vals.items()}
res = {'kernel': kname, 'dispatches_per_counter': {k: len(v) for k, v in vals.items()},
       'counters_mean_per_dispatch': mean,
       'profiled_avg_duration_ms': sum(durs) / max(1, len(durs)) / 1e6, 'config': config}
if 'FETCH_SIZE' in mean and 'WRITE_SIZE' in mean:
    res['hbm_bytes_per_launch'] = (2 * mean['FETCH_SIZE'] + mean['WRITE_SIZE']) * 1024
    res['hbm_read_bytes_per_launch'] = 2 * mean['FETCH_SIZE'] * 1024
    res['hbm_write_bytes_per_launch'] = mean['WRITE_SIZE'] * 1024
if 'GRBM_GUI_ACTIVE' in mean:
    res['effective_clock_ghz'] = mean['GRBM_GUI_ACTIVE'] / 8 / (res['profiled_avg_duration_ms'] * 1e-3) / 1e9
json.dump(res, open(out, 'w'), indent=1)
print(json.dumps({k: res[k] for k in res if k not in ('counters_mean_per_dispatch',)}, indent=1))
