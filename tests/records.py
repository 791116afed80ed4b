"""numpy writer of vio_ba record bytes (include/vio360.h, VIO_BA_RECORD_VERSION 1) — TEST
INFRASTRUCTURE: lets the CPU (gloo) rehearsal of the config-4 gather pack oracle results in the same
layout the device pack kernel writes; the product decoder is libvio360's vio_ba_record_unpack."""
import numpy as np

VERSION = 1


def layout(K, L, N):
    o = {"si": 16, "sd": 48, "T": 80}
    o["lm"] = o["T"] + 96 * K
    o["vel"] = o["lm"] + 24 * L
    o["bias"] = o["vel"] + 24 * K
    o["outl"] = o["bias"] + 48
    o["bad"] = o["outl"] + N
    o["total"] = (o["bad"] + L + 15) & ~15
    return o


def pack(r, K, L, N, nbytes=None):
    lo = layout(K, L, N)
    rec = np.zeros(nbytes or lo["total"], np.uint8)
    rec[:16] = np.array([K, L, N, VERSION], np.int32).view(np.uint8)
    si = [r["success"], r["termination"], r["iterations"], r["num_successful_steps"], r["num_unsuccessful_steps"],
          r["num_inliers"], r["num_outliers"], r["num_bad_lm"]]
    rec[lo["si"]:lo["si"] + 32] = np.array(si, np.int32).view(np.uint8)
    rec[lo["sd"]:lo["sd"] + 32] = np.array([r["initial_cost"], r["final_cost"], r["fixed_cost"], 0.0]).view(np.uint8)
    T = np.concatenate([np.concatenate([r["T_wb"][k, :3, :3].reshape(-1), r["T_wb"][k, :3, 3]]) for k in range(K)])
    rec[lo["T"]:lo["lm"]] = T.astype(np.float64).view(np.uint8)
    rec[lo["lm"]:lo["vel"]] = np.ascontiguousarray(r["lm_xyz"], np.float64).reshape(-1).view(np.uint8)
    rec[lo["vel"]:lo["bias"]] = np.ascontiguousarray(r["vel"], np.float64).reshape(-1)[:3 * K].view(np.uint8)
    rec[lo["bias"]:lo["outl"]] = np.concatenate([r["bg"], r["ba"]]).astype(np.float64).view(np.uint8)
    rec[lo["outl"]:lo["bad"]] = r["obs_outlier"][:N]
    rec[lo["bad"]:lo["bad"] + L] = r["lm_bad"][:L]
    return rec
