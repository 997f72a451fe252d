"""Print the key figures of a bench.py JSON line: python tools/summarise_line.py LINE.json"""
import json
import sys

with open(sys.argv[1]) as fh:
    d = json.loads([l for l in fh if l.lstrip().startswith("{")][-1])
r = d["roofline"]
cpu = d.get("cpu_baseline") or {}
sp = d.get("step_split") or {}
print(f"{d['config'].get('launch_mode')} N={d['n_gpus']} value {d['value']:.4g} {d['unit']} "
      f"ms/step {d['ms_per_step']:.3f} launch {r['avg_launch_ms']:.4f} ms frac {r['frac']:.4f} "
      f"probe {r.get('write_probe_gbs') or 0:.0f} GB/s of-probe {r.get('frac_of_write_probe') or 0:.3f} "
      f"sclk {d['sclk'].get('mean_mhz', 0):.0f} cpu {cpu.get('value', 0):.3g} "
      f"tail {sp.get('exposed_tail_ms', 0):.3f} ms | {d['parity']} | rows: {d.get('parity_rows')}"
      + (f" | slots fastest/slowest {r['per_slot']['fastest_over_slowest']:.3f}" if r.get('per_slot') else ""))
st = d.get("stages_ms")
if st:
    print("  stages ms: " + ", ".join(f"{k} {v:.3f}" for k, v in st.items() if k != "note")
          + f" | valu {((d.get('valu_roofline') or {}).get('frac') or 0):.3f}")
n = d.get("c2match")
if n:
    print(f"  c2match: {n['value']:.4g} {n['unit']} ms/step {n['ms_per_step']:.3f} | "
          + ", ".join(f"{k} {v:.3f}" for k, v in n["stages_ms"].items() if k != "note")
          + f" | {n['parity']} | wall {n.get('wall_s', 0):.1f} s")
