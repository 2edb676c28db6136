"""GPU timeline of a bench run from a rocprofv3 kernel trace (csv): the timed steps are the last
--steps stretches between optimizer launches (adam_ema_dev_kernel ends a step); per step the wall
span, the busy time (union of all kernel intervals), the idle gaps > 20 us and the time two or more
kernels overlap (side stream).  Usage: python tools/timeline.py kernel_trace.csv [--steps 10]"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument('trace')
ap.add_argument('--steps', type=int, default=10)
args = ap.parse_args()
rows = list(csv.DictReader(open(args.trace)))
ks = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'], r.get('Queue_Id', ''))
            for r in rows)
ends = [e for s, e, n, q in ks if 'adam_ema' in n]
bounds = ends[-(args.steps + 1):]
tot_busy = tot_span = 0
for a, b in zip(bounds, bounds[1:]):
    seg = [(s, e, n, q) for s, e, n, q in ks if s >= a and s < b]
    span = b - a
    busy = 0
    cur_s = cur_e = None
    gaps = []
    for s, e, n, q in seg:
        if cur_e is None:
            cur_s, cur_e = s, e
            if s - a > 20000:
                gaps.append((s - a, 'start', n[:40]))
        elif s > cur_e:
            busy += cur_e - cur_s
            if s - cur_e > 20000:
                gaps.append((s - cur_e, prev[:40], n[:40]))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev = n
    if cur_e is not None:
        busy += cur_e - cur_s
    ksum = sum(e - s for s, e, n, q in seg)
    queues = sorted(set(q for s, e, n, q in seg))
    tot_busy += busy
    tot_span += span
    print(f'step span {span / 1e6:.2f} ms  busy {busy / 1e6:.2f} ms  idle {(span - busy) / 1e6:.2f} ms  kernel sum '
          f'{ksum / 1e6:.2f} ms (overlap {(ksum - busy) / 1e6:.2f})  launches {len(seg)}  queues {queues}  '
          f'gaps>20us {len(gaps)} = {sum(g[0] for g in gaps) / 1e6:.2f} ms')
    for g in sorted(gaps, reverse=True)[:6]:
        print(f'    gap {g[0] / 1e3:.0f} us after {g[1]} before {g[2]}')
print(f'mean: span {tot_span / 1e6 / max(1, len(bounds) - 1):.2f} ms, busy {tot_busy / 1e6 / max(1, len(bounds) - 1):.2f} ms')
