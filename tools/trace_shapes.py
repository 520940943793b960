"""Group the last N optimizer steps of a rocprofv3 kernel-trace CSV by (kernel, grid): count, avg us."""
import csv, collections, sys
path, nsteps = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2
pat = sys.argv[3] if len(sys.argv) > 3 else ""
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
opt = [r for r in rows if 'multi_tensor_apply' in r['Kernel_Name'] or 'FusedAdam' in r['Kernel_Name'] or 'adamw_kernel' in r['Kernel_Name']]
ends, steps, last = sorted(set(int(r['End_Timestamp']) for r in opt)), [], None
for e in ends:
    if last is None or e - last > 3e6:
        steps.append(e)
    last = e
s_a, s_b = steps[-1 - nsteps], steps[-1]
agg, cnt = collections.defaultdict(float), collections.Counter()
for r in rows:
    s = int(r['Start_Timestamp'])
    if s_a < s <= s_b and pat in r['Kernel_Name']:
        k = r['Kernel_Name'].replace('(anonymous namespace)::', '')
        k = (k.split('(')[0] if not k.startswith('void') else k[:70])[:70]
        key = (k, r['Grid_Size_X'], r['Grid_Size_Y'], r['Grid_Size_Z'], r['Workgroup_Size_X'])
        agg[key] += int(r['End_Timestamp']) - s
        cnt[key] += 1
for k, v in sorted(agg.items(), key=lambda x: -x[1]):
    print(f"{v / nsteps / 1e3:8.1f} us/step n={cnt[k] / nsteps:4.0f} avg={v / cnt[k] / 1e3:7.1f}us grid={k[1]}x{k[2]}x{k[3]} wg={k[4]} {k[0]}")
