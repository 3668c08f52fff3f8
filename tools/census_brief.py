"""One line per (call, kernel) of a tools/census.py JSON: span, wave lifetimes, start offsets, residency."""
import json
import sys

for f in sys.argv[1:]:
    d = json.load(open(f))
    print("==", f, d.get("env"))
    for k, v in d["kernels"].items():
        print("%-18s w%6d st%8.1f end%8.1f span%7.1f life%-20s off%-22s res%5d wps%d" % (
            k, v["waves"], v["start_us"], v["end_us"], v["span_us"], v["life_p50_p90_max"],
            v["start_off_p50_p90_max"], v["max_resident"], v["waves_per_simd_max"]))
    for k, v in d["parsers"].items():
        print(k, "late p50/p99/max", v["late_start_us_p50_p99_max"], "n_late>20us", v["n_late_over_20us"],
              "hist", v["parsers_per_simd_hist"])
