#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc passes taken over `bench.py --config X` into the stamped profile
profiles/pmc/<config_key>.json that bench.py attaches to its `roofline` (traffic, VALU).

Each pass is its own rocprofv3 run (tools/gpu_pmc_bench.sh): FETCH_SIZE, WRITE_SIZE, and one SQ
group.  Per kernel the counter is averaged over its dispatches (all dispatches of a kernel in a
bench run have the same shape).  Corrections (MI355X_MICROARCH.md, "HBM [CDNA4]"): FETCH_SIZE is
in KiB and on gfx950 reports half the bytes of wide coalesced reads -> read bytes =
2 * 1024 * FETCH_SIZE (an upper bound for narrow / gathered reads, which the guide leaves
uncalibrated); WRITE_SIZE is in KiB, exact for streaming stores -> 1024 * WRITE_SIZE.

usage: pmc_bench.py CONFIG_KEY OUT.json PASS_DIR [PASS_DIR ...]
The profile is stamped with bench.source_hash() (the library sources it was taken on): bench.py
ignores a profile whose stamp differs from the current sources.
"""
import collections
import csv
import glob
import json
import os
import sys

NAMES = {"k12_fwd_grad": "K12_photometric_fwd_grad", "k0_unwarped": "K0_unwarped", "k_sig_sum": "sig_sum",
         "k_grad_finish": "grad_finish", "k_finalize": "finalize", "k_pose_reduce": "pose_grad_reduce",
         "k1_forward": "K1_photometric_fwd", "k2_backward": "K2_photometric_bwd",
         "k_p3d_fwd_cl": "p3d_fwd_cl", "k_p3d_bwd_x_cl": "p3d_bwd_x_cl", "k_p3d_bwd_w_mfma": "p3d_bwd_w_mfma",
         "k_p3d_reduce_w": "p3d_reduce_w", "k_p3d_fwd": "p3d_fwd", "k_p3d_bwd_x": "p3d_bwd_x", "k_p3d_bwd_w": "p3d_bwd_w", "k_adam": "adam",
         "k_gn_fwd_stats": "gn_fwd_stats", "k_gn_fwd_apply": "gn_fwd_apply", "k_gn_bwd_stats": "gn_bwd_stats",
         "k_gn_bwd_apply": "gn_bwd_apply", "k_bias_act_fwd": "bias_act_fwd", "k_bias_act_bwd": "bias_act_bwd",
         "k_cols_finish": "cols_finish", "k_upcat_fwd": "upcat_fwd", "k_upcat_bwd": "upcat_bwd",
         "k_gnp_fwd_stats": "gnp_fwd_stats", "k_gnp_fwd_apply": "gnp_fwd_apply", "k_gnp_bwd_stats": "gnp_bwd_stats",
         "k_gnp_bwd_apply": "gnp_bwd_apply", "k_gnr_fwd": "gnr_fwd", "k_gnr_bwd": "gnr_bwd", "k_gnr_params": "gnr_params",
         "k_bnr_fwd": "bnr_fwd", "k_bnr_bwd": "bnr_bwd", "k_pc_conv": "pc_conv", "k_pc_wgrad": "pc_wgrad"}


def label(kernel):
    for key, name in NAMES.items():
        if key in kernel:
            return name
    return None


def read_pass(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in files:
        for r in csv.DictReader(open(f)):
            lab = label(r["Kernel_Name"])
            if lab is None:
                continue
            # one row per (dispatch, counter); the value is already summed over the device
            acc[lab][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def main():
    key, out = sys.argv[1], sys.argv[2]
    kernels = collections.defaultdict(dict)
    for d in sys.argv[3:]:
        for lab, ctrs in read_pass(d).items():
            for c, vals in ctrs.items():
                kernels[lab][c] = sum(vals) / len(vals)
                kernels[lab].setdefault("dispatches", {})[c] = len(vals)
    for lab, k in kernels.items():
        rd = 2 * 1024 * k["FETCH_SIZE"] if "FETCH_SIZE" in k else None
        wr = 1024 * k["WRITE_SIZE"] if "WRITE_SIZE" in k else None
        k["read_bytes"], k["write_bytes"] = rd, wr
        k["hbm_bytes"] = (rd + wr) if rd is not None and wr is not None else None
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    res = {"config_key": key, "source_hash": bench.source_hash(),
           "source": "rocprofv3 --pmc over bench.py (one pass per counter group, tools/gpu_pmc_bench.sh)",
           "correction": "read = 2*1024*FETCH_SIZE (gfx950 half-count of wide reads), write = 1024*WRITE_SIZE",
           "kernels": kernels}
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps({k: {c: v for c, v in d.items() if c in ("hbm_bytes", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU")}
                      for k, d in kernels.items()}, indent=1))


if __name__ == "__main__":
    main()
