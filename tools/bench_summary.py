"""Summary of a bench.py JSON line (the last '{' line of a log): headline, legs, CPU baselines."""
import json
import sys

d = json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
print(f"headline {d['value']:.0f} {d['unit']}  ms/step {d['ms_per_step']:.3f}  roofline frac {d['roofline']['frac']:.4f} "
      f"kernel {d['roofline']['kernel_avg_ms']:.3f} ms")
s = d["single_window"]
print(f"single window {s['iters_per_s_wall']:.0f} it/s (kernel {s['kernel_ms']:.3f} ms / 10 it), with transfer "
      f"{s['iters_per_s_with_transfer']:.0f}; vs cpu 1t {s['vs_cpu_1t']}, 4t {s['vs_cpu_4t']}")
c4 = d.get("config4_strong") or {}
print(f"config4 strong (1 GPU) {c4.get('value', 0):.0f} ms {c4.get('ms_per_step', 0):.3f}; shard32 {d['config4_shard32']}")
c2 = d.get("config2") or {}
if c2:
    print(f"config2 {c2['value']:.0f} it/s kernel {c2['kernel_ms']:.3f} ms, batched {c2['batched']}, cpu {c2['cpu_baseline'] and c2['cpu_baseline']['by_threads']}")
k = d.get("erp_klt") or {}
if k:
    print(f"klt {k['value']:.0f} Mpx/s device {k['device_ms_per_step']:.4f} ms stages {k['stage_ms']} frac {k['roofline']['frac']:.4f}")
g = d.get("global_ba") or {}
if g:
    print(f"global BA {g['ms_per_iteration']:.3f} ms/it frac {g['roofline']['frac']:.4f} traffic {g['roofline']['traffic']}")
c = d.get("cpu_baseline") or {}
if c:
    print(f"cpu single {c['single_window_threads']} config4 {c['config4_windows_parallel']}")
