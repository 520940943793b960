"""Per-step kernel-time breakdown from a rocprofv3 kernel-trace CSV (last N optimizer steps)."""
import csv, collections, sys
path = sys.argv[1]
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
opt = [r for r in rows if 'multi_tensor_apply' in r['Kernel_Name'] or 'FusedAdam' in r['Kernel_Name'] or 'adamw_kernel' in r['Kernel_Name']]
ends = sorted(set(int(r['End_Timestamp']) for r in opt))
steps, last = [], None
for e in ends:
    if last is None or e - last > 3e6:
        steps.append(e)
    last = e
s_a, s_b = steps[-1 - nsteps], steps[-1]
agg, cnt = collections.defaultdict(float), collections.Counter()
for r in rows:
    s = int(r['Start_Timestamp'])
    if s_a < s <= s_b:
        k = r['Kernel_Name']
        k = k.replace('(anonymous namespace)::', '')
        key = (k.split('(')[0] if not k.startswith('void') else k[:80])[:95]
        agg[key] += int(r['End_Timestamp']) - s
        cnt[key] += 1
tot = sum(agg.values())
print(f"kernel busy {tot / nsteps / 1e6:.2f} ms/step, wall {(s_b - s_a) / nsteps / 1e6:.2f} ms/step")
for k, v in sorted(agg.items(), key=lambda x: -x[1])[:int(sys.argv[3]) if len(sys.argv) > 3 else 40]:
    print(f"{v / nsteps / 1e3:9.1f} us/step {100 * v / tot:5.1f}%  n={cnt[k] / nsteps:5.0f}  avg={v / cnt[k] / 1e3:7.1f}us  {k}")
