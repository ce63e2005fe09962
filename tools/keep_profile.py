#!/usr/bin/env python3
"""Copy a profile's judged artifacts from gpurun_out/ into profiles/ (tracked).

Usage: keep_profile.py <gpurun_out/name> <tag> [--pmc-config c3]
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_summary.json       per-kernel averages (all launches and timed window)
  profiles/pmc_<config>.json        HBM bytes per launch of the step kernel, keyed on the
                                    library's build id (bench.py reads it for
                                    roofline.traffic only when the build matches)
"""
import glob
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(src, tag, cfg=None):
    dst = os.path.join(REPO, "profiles")
    os.makedirs(dst, exist_ok=True)
    st = glob.glob(os.path.join(src, "kt", "**", "*kernel_stats.csv"), recursive=True)[0]
    shutil.copy(st, os.path.join(dst, tag + "_kernel_stats.csv"))
    summ = json.load(open(os.path.join(src, "summary.json")))
    json.dump(summ, open(os.path.join(dst, tag + "_summary.json"), "w"), indent=1, sort_keys=True)
    if cfg:
        # the bench's step kernel: the one launched for every timed step (a few steps
        # outside the timed window -- the changed-rows measurement, views of a first
        # step -- may run another instance)
        step = [k for k in summ["kernels"] if "k_env_step" in k]
        if not step:
            raise SystemExit("no step kernel in the profile")
        k = max(step, key=lambda n: summ["kernels"][n].get("calls", 0))
        d = summ["kernels"][k]
        lk = d.get("last_k", {})
        bid_path = os.path.join(REPO, "safelife-k2_amd", "safelife_amd", "_native",
                                "build_id.txt")
        bid = open(bid_path).read().strip() if os.path.exists(bid_path) else None
        rec = {"kernel": k, "profile": tag, "build_id": bid,
               "hbm_bytes_per_launch": lk.get("hbm_bytes_per_launch", d.get("hbm_bytes_per_launch")),
               "hbm_read_bytes": lk.get("hbm_read_bytes", d.get("hbm_read_bytes")),
               "hbm_write_bytes": lk.get("hbm_write_bytes", d.get("hbm_write_bytes")),
               "avg_ns_timed_window": d.get("last_k_avg_ns"), "avg_ns_all": d.get("avg_ns"),
               "note": "FETCH_SIZE x2 + WRITE_SIZE (MI355X_MICROARCH.md HBM section), averaged "
                       "over the bench's timed window (last %s launches)" % summ.get("last_k")}
        json.dump(rec, open(os.path.join(dst, "pmc_%s.json" % cfg), "w"), indent=1)
        print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    a = sys.argv[1:]
    cfg = None
    if "--pmc-config" in a:
        i = a.index("--pmc-config")
        cfg = a[i + 1]
        del a[i:i + 2]
    main(a[0], a[1], cfg)
