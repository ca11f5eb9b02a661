"""Summarise a tools/profile.sh run: kernel-trace durations + PMC counters
per hbx kernel, for the largest dispatch shape of each kernel (the bench's
step launches).  HBM bytes follow MI355X_MICROARCH.md (HBM/rocprofv3):
FETCH_SIZE and WRITE_SIZE are collected in separate passes and are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced stream, so
hbm_read = 2 * FETCH_SIZE * 1024 and hbm_write = WRITE_SIZE * 1024.

usage: python tools/pmc_summary.py gpurun_out/prof_<tag> [--jobs 128 --N 1024 --out profiles/pmc_latest.json]
"""
import argparse
import csv
import json
import os
import re
from collections import defaultdict

KERNELS = ("k_rowfwd", "k_col", "k_rowinv", "k_psf_eval", "k_psf_commit")


def short(name):
    m = re.search(r"hbx::(k_[a-z_]+)", name)
    if not m:
        return None
    k = m.group(1)
    return k[:-2] if k.endswith("_d") else k     # k_rowinv_d (r03's direct-load variant) is the k_rowinv pass


def load_counters(path):
    """{(kernel, grid): {counter: [values per dispatch]}}"""
    out = defaultdict(lambda: defaultdict(list))
    per_dispatch = defaultdict(dict)
    with open(path) as f:
        for row in csv.DictReader(f):
            k = short(row["Kernel_Name"])
            if k is None:
                continue
            key = (k, int(row["Grid_Size"]))
            per_dispatch[(key, row["Dispatch_Id"])][row["Counter_Name"]] = float(row["Counter_Value"])
            per_dispatch[(key, row["Dispatch_Id"])]["_vgpr"] = int(row["VGPR_Count"])
            per_dispatch[(key, row["Dispatch_Id"])]["_lds"] = int(row["LDS_Block_Size"])
    for (key, _), cs in per_dispatch.items():
        for c, v in cs.items():
            out[key][c].append(v)
    return out


def load_trace(path):
    out = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            k = short(row["Kernel_Name"])
            if k is None:
                continue
            g = int(row["Grid_Size_X"]) * int(row["Grid_Size_Y"]) * int(row["Grid_Size_Z"])
            out[(k, g)].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--jobs", type=int, default=128)
    ap.add_argument("--N", type=int, default=1024)
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    N, P = a.N, a.P
    alg = {"k_rowfwd": P * N * N // 8 + P * N * N * 4, "k_col": P * N * N * 12,
           "k_rowinv": P * N * N * 8 + N * N * 4, "k_psf_eval": 16 * N * N,
           "k_psf_commit": 24 * N * N}   # commit: per ACCEPTED job
    trace = load_trace(os.path.join(a.dir, "trace", "run_kernel_trace.csv"))
    cnt = {}
    for sub in ("fetch", "write", "sq", "lds"):
        p = os.path.join(a.dir, sub, "run_counter_collection.csv")
        if os.path.exists(p):
            for key, cs in load_counters(p).items():
                cnt.setdefault(key, {}).update(cs)
    res = {"N": N, "jobs_per_launch": a.jobs, "source": a.dir, "kernels": {}}
    for k in KERNELS:
        keys = [key for key in trace if key[0] == k]
        if not keys:
            continue
        key = max(keys, key=lambda x: x[1])          # largest grid = step launch
        durs = trace[key]
        avg = sum(durs) / len(durs)
        cs = cnt.get(key, {})
        mean = lambda c: (sum(cs[c]) / len(cs[c])) if c in cs else None  # noqa: E731
        fetch, write = mean("FETCH_SIZE"), mean("WRITE_SIZE")
        hbm = None
        if fetch is not None and write is not None:
            hbm = 2.0 * fetch * 1024 + write * 1024
        info = {"grid": key[1], "avg_ms": avg * 1e3, "dispatches": len(durs),
                "alg_bytes_per_launch": alg[k] * a.jobs,
                "alg_GBs": alg[k] * a.jobs / avg / 1e9,
                "hbm_read_bytes": None if fetch is None else 2.0 * fetch * 1024,
                "hbm_write_bytes": None if write is None else write * 1024,
                "hbm_bytes_per_launch": hbm,
                "hbm_GBs": None if hbm is None else hbm / avg / 1e9,
                "jobs_per_launch": float(a.jobs), "N": N,
                "vgpr": mean("_vgpr"), "lds_bytes": mean("_lds")}
        wc = mean("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                      "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT",
                      "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS", "GRBM_GUI_ACTIVE"):
                if mean(c) is not None:
                    info[c] = mean(c)
            info["frac_wait_any"] = mean("SQ_WAIT_ANY") / wc if mean("SQ_WAIT_ANY") else None
            info["frac_wait_inst"] = mean("SQ_WAIT_INST_ANY") / wc if mean("SQ_WAIT_INST_ANY") else None
            info["frac_active"] = mean("SQ_ACTIVE_INST_ANY") / wc if mean("SQ_ACTIVE_INST_ANY") else None
        if k == "k_psf_commit":
            # only accepted envs rewrite their plane: the per-launch algorithmic bytes depend on
            # the accept count (bench.py charges the accepted jobs); the PMC bytes are the truth here
            info["alg_bytes_per_launch"] = None
            info["alg_GBs"] = None
            info["note"] = "24 N^2 B per ACCEPTED job; see hbm_bytes_per_launch / bench.py passes"
        res["kernels"][k] = info
    txt = json.dumps(res, indent=1)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
