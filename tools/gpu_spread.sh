# Run-to-run spread of the C3 bench on one box, with clocks and hwmon
# temperatures recorded in each line (attribution of the spread)
set -o pipefail
mkdir -p gpurun_out/spread
for rnd in 1 2 3 4 5; do
  timeout -k 10 240 python bench.py --workload c3 --steps ${STEPS:-10} --warmup 2 --cpu-seconds 0 > gpurun_out/spread/r${rnd}.json 2> gpurun_out/spread/r${rnd}.err || { tail -5 gpurun_out/spread/r${rnd}.err; exit 1; }
  python - gpurun_out/spread/r${rnd}.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d["roofline"]
t = d.get("temperature") or {}
print("%.4g pairs/s launch %.3f ms probe %.0f of-probe %.3f sclk %s mclk %s fclk %s temps %s" % (
    d["value"], r["avg_launch_ms"], r["write_probe_gbs"], r["frac_of_write_probe"],
    d["sclk"].get("mean_mhz"), d["mclk"].get("mean_mhz"), d["fclk"].get("mean_mhz"),
    {k: (v["first_c"], v["last_c"]) for k, v in t.items()}))
PY
done
