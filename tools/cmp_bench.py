"""Side-by-side bench lines of gpurun_out/<tag>/bench_*.json for A/B runs:
    python tools/cmp_bench.py r05s r05t"""
import json
import sys

for f in ["dense", "collision", "share", "fov", "fov_slack"]:
    for t in sys.argv[1:]:
        try:
            d = json.loads(open(f"gpurun_out/{t}/bench_{f}.json").read().strip().splitlines()[-1])
        except Exception as e:  # noqa: BLE001 (a missing line is reported, not fatal)
            print(f"{f:10s} {t:6s} ERR {e}")
            continue
        r = d.get("roofline", {})
        print(f"{f:10s} {t:6s} value {d['value']:.4g} ms/step {d['ms_per_step'] * 1000:.2f} us "
              f"kernel {r.get('kernel_avg_us')} events {r.get('kernel_event_bracket_avg_us')} "
              f"single {d.get('single_qp_latency_ms', {}).get('median')}")
