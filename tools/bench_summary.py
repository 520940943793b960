"""One-screen summary of bench.py JSON lines: value, ms/step, dominant kernel, per-kernel table.
    python tools/bench_summary.py <bench.json> [...] [--top N]"""
import json
import sys


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    top = 14
    if "--top" in sys.argv:
        top = int(sys.argv[sys.argv.index("--top") + 1])
        args = [a for a in args if a != str(top)]
    for path in args:
        lines = [l for l in open(path).read().strip().splitlines() if l.startswith("{")]
        if not lines:
            print(path, "no JSON line")
            continue
        r = json.loads(lines[-1])
        roof = r.get("roofline") or {}
        print(f"{path}: {r['value']} {r['unit']}  {r['ms_per_step']} ms/step  dominant {roof.get('kernel')} "
              f"frac {roof.get('frac')} step_frac {roof.get('step_frac')} traffic {roof.get('traffic')}")
        for k in (roof.get("kernels") or [])[:top]:
            print(f"   {k['kernel']:<18} {k['us_per_step']:>9.1f} us/step  {k['launches_per_step']:>4} launches  "
                  f"frac {k['frac']}")
        if r.get("cpu_baseline"):
            print("   cpu_baseline", r["cpu_baseline"].get("value"), r["cpu_baseline"].get("sample"))


if __name__ == "__main__":
    main()
