"""CPU checks of the C-ABI boundary: libvio360.so loads, exports every entry point include/vio360.h
declares, and the ctypes mirror (abi.py) is byte-identical to the header structs."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "vio360.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\**\s*([a-z_0-9]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_library_exports_every_header_symbol(vio):
    lib = C.CDLL(vio.LIB_PATH)
    names = header_functions()
    assert len(names) >= 20, names
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # the Python wrapper's export list is the header's
    assert set(vio.EXPORTS) <= set(names)


def test_abi_version(vio):
    assert vio.lib().vio_abi_version() == 4  # 4: VIO_BA_PROF_SLOTS 24 -> 32


STRUCTS = {
    "vio_pose": ("VioPose", ["R", "t"]),
    "vio_preint": ("VioPreint", ["delta_R", "delta_V", "delta_P", "J_Rg", "cov9", "gyro_bias", "accel_bias", "dt_total"]),
    "vio_ba_problem": ("VioBaProblem", ["variant", "num_kf", "cols", "info", "chi2_threshold", "T_cb", "T_wb_init",
                                        "kf_const", "lm_xyz", "obs_uv", "preint", "vel", "bg", "gravity",
                                        "max_iterations", "fixed_iterations", "num_rounds"]),
    "vio_ba_summary": ("VioBaSummary", ["success", "num_bad_lm", "initial_cost", "fixed_cost"]),
    "vio_ba_output": ("VioBaOutput", ["T_wb", "lm_xyz", "obs_outlier", "summary", "trace", "trace_cap"]),
    "vio_ba_iteration": ("VioBaIteration", ["iteration", "step_is_valid", "step_is_successful", "cost",
                                            "cost_change", "gradient_max_norm", "step_norm", "relative_decrease",
                                            "trust_region_radius", "model_cost_change"]),
    "vio_imu_data": ("VioImuData", ["timestamp", "ax", "az", "gx", "gz"]),
    "vio_imu_noise": ("VioImuNoise", ["gyro_noise", "accel_bias_noise"]),
    "erp_klt_params": ("ErpKltParams", ["win", "max_level", "epsilon", "min_eig_threshold"]),
    "erp_tracker_params": ("ErpTrackerParams", ["ransac_iters", "ransac_seed", "quality", "min_dist",
                                                "boundary_margin", "polar_ratio"]),
    "vio_map_view": ("VioMapView", ["num_frames", "num_mappoints", "frame_Twb", "frame_Tcb", "feat_begin", "feat_uv",
                                    "feat_valid", "feat_mp", "mp_key", "mp_bad", "mp_marg", "mp_pos", "mp_obs_begin",
                                    "mp_obs_frame", "mp_obs_feat", "width", "height", "boundary_margin"]),
    "vio_ba_gather_out": ("VioBaGatherOut", ["status", "num_lm", "num_obs", "cap_lm", "cap_obs", "lm_mp", "lm_const",
                                             "lm_marg", "lm_xyz", "obs_kf", "obs_lm", "obs_uv", "obs_feat", "kf_const",
                                             "kf_in_problem", "T_wb_init", "T_cb"]),
    "vio_mono_init_params": ("VioMonoInitParams", ["width", "height", "min_features", "ransac_iterations",
                                                   "ransac_threshold", "max_reprojection_error"]),
    "vio_mono_init_result": ("VioMonoInitResult", ["status", "best_hypothesis", "num_inliers", "pose_candidate",
                                                   "candidate_good", "num_triangulated", "num_valid",
                                                   "mean_reproj_error", "scale_factor", "E", "R", "t"]),
    "vio_window_frame": ("VioWindowFrame", ["frame_id", "num_features", "width", "T_wb", "T_bc", "feature_id", "uv",
                                            "bearing", "valid", "mappoint", "track_begin", "track_frame",
                                            "track_feat"]),
    "vio_window_kf_stats": ("VioWindowKfStats", ["obs_added", "transferred", "deleted", "removed_frame",
                                                 "num_keyframes"]),
    "vio_window_mappoint_info": ("VioWindowMappointInfo", ["pos", "bad", "marginalized", "triangulated",
                                                           "reference_frame", "num_observations"]),
    "vio_ba_map_update": ("VioBaMapUpdate", ["frame_Twb", "frame_set", "frame_vel", "bias", "mp_pos", "mp_set",
                                             "mp_set_bad", "success", "num_inliers", "num_outliers",
                                             "num_poses_optimized", "num_points_optimized", "num_iterations",
                                             "initial_cost", "final_cost"]),
}


def test_struct_layout_matches_header(vio, tmp_path):
    lines = ["#include <stdio.h>", "#include <stddef.h>", f'#include "{HEADER}"', "int main(void){"]
    for cs, (_, fields) in STRUCTS.items():
        lines.append(f'printf("{cs} sizeof %zu\\n", sizeof({cs}));')
        for f in fields:
            lines.append(f'printf("{cs} {f} %zu\\n", offsetof({cs}, {f}));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-o", str(exe), str(src)])
    out = subprocess.check_output([str(exe)]).decode().split("\n")
    got = {}
    for ln in out:
        if ln:
            s, f, v = ln.split()
            got[(s, f)] = int(v)
    for cs, (py, fields) in STRUCTS.items():
        cls = getattr(vio.abi, py)
        assert C.sizeof(cls) == got[(cs, "sizeof")], cs
        for f in fields:
            assert getattr(cls, f).offset == got[(cs, f)], (cs, f)


def test_no_device_fails_loudly(vio):
    """Without a GPU the product path must raise (there is no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(vio.VioError):
        vio.Context(0)


def test_frontend_params_layout(vio, tmp_path):
    src = tmp_path / "fe.c"
    fields = ["max_features", "min_distance", "quality_level", "boundary_margin", "grid_cols", "grid_rows",
              "max_features_per_grid", "remove_clustered", "clustered_std_ratio", "ransac_seed"]
    lines = ["#include <stdio.h>", "#include <stddef.h>", f'#include "{HEADER}"', "int main(void){",
             'printf("%zu\\n", sizeof(erp_frontend_params));']
    lines += [f'printf("%zu\\n", offsetof(erp_frontend_params, {f}));' for f in fields]
    src.write_text("\n".join(lines + ["return 0;}"]))
    subprocess.check_call(["gcc", "-o", str(tmp_path / "fe"), str(src)])
    out = [int(x) for x in subprocess.check_output([str(tmp_path / "fe")]).split()]
    cls = vio.abi.ErpFrontendParams
    assert out[0] == C.sizeof(cls)
    assert out[1:] == [getattr(cls, f).offset for f in fields]


def _record(K=3, L=5, N=7):
    import numpy as np
    import records
    rng = np.random.default_rng(4)
    T = np.tile(np.eye(4), (K, 1, 1))
    T[:, :3, 3] = rng.normal(size=(K, 3))
    r = {"success": 1, "termination": 0, "iterations": 4, "num_successful_steps": 3, "num_unsuccessful_steps": 1,
         "num_inliers": N - 1, "num_outliers": 1, "num_bad_lm": 0, "initial_cost": 2.0, "final_cost": 1.0,
         "fixed_cost": 0.0, "T_wb": T, "lm_xyz": rng.normal(size=(L, 3)), "vel": rng.normal(size=(K, 3)),
         "bg": rng.normal(size=3), "ba": rng.normal(size=3), "obs_outlier": (np.arange(N) == 2).astype(np.uint8),
         "lm_bad": np.zeros(L, np.uint8)}
    return r, records.pack(r, K, L, N)


def test_record_unpack_round_trip_and_rejects_malformed(vio):
    """vio_ba_record_unpack (host decoder of the all-gathered records) takes the record's length and
    rejects a header whose K/L/N layout overruns it, a short record and a bad version (records come
    from other ranks)."""
    import numpy as np
    r, rec = _record()
    out = vio.unpack_record(rec)
    assert np.array_equal(out["lm_xyz"], r["lm_xyz"]) and out["iterations"] == 4
    assert np.array_equal(out["obs_outlier"], r["obs_outlier"])
    lib = vio.lib()
    o = vio.BaOutput(3, 5, 7)
    buf = np.ascontiguousarray(rec)
    p = buf.ctypes.data
    assert lib.vio_ba_record_unpack(p, buf.size, C.byref(o.c)) == 0
    assert lib.vio_ba_record_unpack(p, buf.size - 1, C.byref(o.c)) == -22  # layout overruns the length
    assert lib.vio_ba_record_unpack(p, 15, C.byref(o.c)) == -22            # shorter than the header
    bad = buf.copy()
    bad[:4] = np.array([1 << 24], np.int32).view(np.uint8)                 # corrupt K
    assert lib.vio_ba_record_unpack(bad.ctypes.data, bad.size, C.byref(o.c)) == -22
    bad = buf.copy()
    bad[12:16] = np.array([99], np.int32).view(np.uint8)                   # unknown version
    assert lib.vio_ba_record_unpack(bad.ctypes.data, bad.size, C.byref(o.c)) == -22
    with pytest.raises(vio.VioError):
        vio.unpack_record(rec[:-16])
