#!/usr/bin/env python
"""profiles/<round>_configs_bench.json: the GPU figures of every BASELINE config
(tools/bench_configs.py, the `configs` step of tools/gpu_check.sh) with the CPU column of each
(tools/cpu_configs.py, the oracle on the same box's host cores) as its `cpu_baseline`, and the
graph-builder line (tools/bench_stag.py) — VERDICT r4 item 7.

  python tools/merge_configs.py r05 gpurun_out/configs.log profiles/r05_cpu_configs.json \
      gpurun_out/stag_bench.json
"""
import json
import sys


def last_json(path):
    line = [ln for ln in open(path) if ln.startswith("{")][-1]
    return json.loads(line)


def main():
    tag, cfg_log, cpu_json, stag_json = sys.argv[1:5]
    gpu = last_json(cfg_log)
    cpu = json.load(open(cpu_json))
    out = {}
    for name, rec in gpu.items():
        r = dict(rec)
        c = cpu.get(name)
        if c is not None:
            r["cpu_baseline"] = c
            if "samples_per_s" in r and c.get("value"):
                r["gpu_over_cpu"] = round(r["samples_per_s"] / c["value"], 1)
        out[name] = r
    out["stag"] = json.load(open(stag_json))
    json.dump(out, open(f"profiles/{tag}_configs_bench.json", "w"), indent=1)
    for k, v in out.items():
        if k == "stag":
            print(k, v["stag_gen"]["pairs_per_s"], "pairs/s")
        else:
            print(k, v.get("ms_per_step"), v.get("samples_per_s"), v.get("cpu_baseline", {}).get("value"))


if __name__ == "__main__":
    main()
