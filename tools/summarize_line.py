"""One-screen summary of a bench.py JSON line: value, step, dominant-kernel launch time and
roofline fraction of the headline and of every leg.   python tools/summarize_line.py <line.json>"""
import json
import sys


def leg(name, d):
    if not d:
        return
    r = d.get('roofline') or {}
    rr = d.get('roofline_rows') or {}
    extra = f" rows {rr.get('avg_launch_ms')} ms frac {rr.get('frac')}" if rr else ''
    print(f"{name:<8} value {d.get('value', 0):.4e} step {d.get('ms_per_step', 0):.4f} ms  "
          f"{r.get('kernel')} {r.get('avg_launch_ms')} ms frac {r.get('frac')} traffic {r.get('traffic')}{extra}")


def main():
    with open(sys.argv[1]) as f:
        line = [ln for ln in f if ln.startswith('{')][-1]
    d = json.loads(line)
    leg('c4', d)
    for k in ('fp64', 'c2', 'c3'):
        leg(k, d.get(k))
    c5 = d.get('c5') or {}
    for k in ('fp32', 'fp64'):
        leg('c5 ' + k, c5.get(k))
    cpu = d.get('cpu_baseline') or {}
    if cpu:
        print(f"cpu      {cpu.get('value', 0):.3e} {cpu.get('unit')} cores {cpu.get('cores')}")


if __name__ == '__main__':
    main()
