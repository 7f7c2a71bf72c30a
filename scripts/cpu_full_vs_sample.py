"""Checks bench.py's bounded CPU-baseline sample against the full batch on the GPU host: the oracle on all
256 objects of config 4 (1 run) vs the default 16-object sample (1 warm-up + median of 3). Prints JSON."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    cfg = bench.CONFIGS[4]
    threads = bench.cpu_threads_default()
    sample = bench.cpu_baseline(cfg, 4, threads, 16, reps=3)
    full = bench.cpu_baseline(cfg, 4, threads, cfg["B"], reps=1)
    print(json.dumps({"threads": threads, "sample_16_objects": sample, "full_256_objects": full,
                      "ratio_full_over_sample": full["value"] / sample["value"]}, indent=1))


if __name__ == "__main__":
    main()
