// ba_map_host.cpp — problem assembly and write-back of the Optimizer entry points (SURVEY §8 a4 and
// the host half of a3) on the flat vio_map_view of the reference's Frame / Feature / MapPoint graph.
//
// Reference: src/optimization/Optimizer.cpp
//   SolvePnP   :83-130 (gather), :272-297 (inlier gate, SetTwb)
//   RunBA      :303-409 (gather, fix first / last), :459-474 (SetTwb every frame, SetPosition of
//              MapPoints neither bad nor marginalised)
//   RunVIBA    :493-636 (gather as RunBA, fix first), :684-712 (+ velocities, shared biases)
//   RunLocalBA :726-851 (gather along MapPoint::GetObservations(), window frames only, pose 0
//              constant when it has a residual, marginalised MapPoints constant), :917-954
//              (SetTwb for frames >= 1 with a residual, SetPosition of every non-marginalised
//              MapPoint — bad ones included)
// Host code: no device work.  The SetBad decision itself (inliers == 0 && outliers >= 2 &&
// !marginalised) is made by the solver (vio_ba_output.lm_bad); this file applies it.
#include <algorithm>
#include <cstring>
#include <numeric>
#include <vector>

#include "vio360.h"

namespace {

// Camera::IsNearBoundary (Camera.cpp:134-139) behind Optimizer::IsNearBoundary (Optimizer.cpp:41-46)
bool near_boundary(const vio_map_view* m, const float* uv) {
    if (m->boundary_margin <= 0) return false;
    const float mg = static_cast<float>(m->boundary_margin);
    return uv[0] < mg || uv[0] > static_cast<float>(m->width) - mg || uv[1] < mg ||
           uv[1] > static_cast<float>(m->height) - mg;
}

void pose_from_f32(const float* T, vio_pose* p) {
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) p->R[3 * r + c] = static_cast<double>(T[4 * r + c]);
        p->t[r] = static_cast<double>(T[4 * r + 3]);
    }
}

// SE3d::matrix().cast<float>()
void pose_to_f32(const vio_pose* p, float* T) {
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) T[4 * r + c] = static_cast<float>(p->R[3 * r + c]);
        T[4 * r + 3] = static_cast<float>(p->t[r]);
    }
    T[12] = T[13] = T[14] = 0.f;
    T[15] = 1.f;
}

bool feature_usable(const vio_map_view* m, int g) {
    // `!feature || !feature->IsValid()` then `!mp || mp->IsBad()`
    if (!m->feat_valid[g]) return false;
    const int mp = m->feat_mp[g];
    return mp >= 0 && mp < m->num_mappoints && !m->mp_bad[mp];
}

bool view_ok(const vio_map_view* m, int variant) {
    if (!m || m->num_frames < 0 || m->num_mappoints < 0) return false;
    if (m->num_frames > 0 && (!m->feat_begin || !m->frame_Twb || !m->frame_Tcb)) return false;
    if (m->num_mappoints > 0 && (!m->mp_key || !m->mp_bad || !m->mp_marg || !m->mp_pos)) return false;
    if (m->num_frames > 0 && m->feat_begin[m->num_frames] > 0 && (!m->feat_uv || !m->feat_valid || !m->feat_mp))
        return false;
    if (variant == VIO_BA_LOCAL && m->num_mappoints > 0 && (!m->mp_obs_begin || !m->mp_obs_frame || !m->mp_obs_feat))
        return false;
    return variant >= VIO_BA_LOCAL && variant <= VIO_PNP;
}

}  // namespace

extern "C" int vio_ba_gather(const vio_map_view* m, int variant, int fix_first, int fix_last, vio_ba_gather_out* g) {
    if (!g || !view_ok(m, variant)) return VIO_EINVAL;
    const int F = m->num_frames;
    g->status = VIO_GATHER_OK;
    g->num_lm = g->num_obs = 0;
    if (F > 0 && (!g->kf_const || !g->kf_in_problem)) return VIO_EINVAL;
    for (int f = 0; f < F; ++f) {
        g->kf_const[f] = 0;
        g->kf_in_problem[f] = 0;
        if (g->T_wb_init) pose_from_f32(m->frame_Twb + 16 * f, &g->T_wb_init[f]);
        if (g->T_cb) pose_from_f32(m->frame_Tcb + 16 * f, &g->T_cb[f]);
    }
    auto push_obs = [&](int f, int lm, int gfeat) -> bool {
        if (g->num_obs >= g->cap_obs || !g->obs_kf || !g->obs_lm || !g->obs_uv || !g->obs_feat) return false;
        const int o = g->num_obs++;
        g->obs_kf[o] = f;
        g->obs_lm[o] = lm;
        g->obs_uv[2 * o] = m->feat_uv[2 * gfeat];
        g->obs_uv[2 * o + 1] = m->feat_uv[2 * gfeat + 1];
        g->obs_feat[o] = gfeat;
        g->kf_in_problem[f] = 1;
        return true;
    };
    auto push_lm = [&](int mp, uint8_t cst) -> bool {
        if (g->num_lm >= g->cap_lm || !g->lm_mp || !g->lm_const || !g->lm_marg || !g->lm_xyz) return false;
        const int l = g->num_lm++;
        g->lm_mp[l] = mp;
        g->lm_const[l] = cst;
        g->lm_marg[l] = m->mp_marg[mp];
        for (int i = 0; i < 3; ++i) g->lm_xyz[3 * l + i] = static_cast<double>(m->mp_pos[3 * mp + i]);
        return true;
    };

    if (variant == VIO_PNP) {
        // one residual block per usable, not-near-boundary feature of the frame; the MapPoint's
        // position is a constant of the factor (one landmark per observation)
        if (F < 1) { g->status = VIO_GATHER_FEW_OBS; return VIO_OK; }
        int n = 0;
        for (int gf = m->feat_begin[0]; gf < m->feat_begin[1]; ++gf)
            if (feature_usable(m, gf) && !near_boundary(m, m->feat_uv + 2 * gf)) ++n;
        if (n < 6) { g->status = VIO_GATHER_FEW_OBS; return VIO_OK; }
        for (int gf = m->feat_begin[0]; gf < m->feat_begin[1]; ++gf) {
            if (!feature_usable(m, gf) || near_boundary(m, m->feat_uv + 2 * gf)) continue;
            const int mp = m->feat_mp[gf];
            if (!push_lm(mp, m->mp_marg[mp]) || !push_obs(0, g->num_lm - 1, gf)) return VIO_EINVAL;
        }
        return VIO_OK;
    }

    if (F < 2) { g->status = VIO_GATHER_FEW_FRAMES; return VIO_OK; }
    // std::set<shared_ptr<MapPoint>> of the usable features' MapPoints, in set order
    std::vector<uint8_t> in_set(m->num_mappoints, 0);
    for (int gf = 0; gf < m->feat_begin[F]; ++gf)
        if (feature_usable(m, gf)) in_set[m->feat_mp[gf]] = 1;
    std::vector<int> order;
    for (int mp = 0; mp < m->num_mappoints; ++mp)
        if (in_set[mp]) order.push_back(mp);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return m->mp_key[a] < m->mp_key[b]; });
    for (size_t i = 1; i < order.size(); ++i)
        if (m->mp_key[order[i]] == m->mp_key[order[i - 1]]) return VIO_EINVAL;  // keys must be unique
    if (order.empty()) { g->status = VIO_GATHER_NO_MAPPOINTS; return VIO_OK; }
    std::vector<int> mp_to_lm(m->num_mappoints, -1);
    for (int mp : order) {
        // RunLocalBA: marginalised MapPoints are SetParameterBlockConstant (:861-869); RunBA / RunVIBA
        // leave them variable (only exempt from SetBad)
        if (!push_lm(mp, variant == VIO_BA_LOCAL ? m->mp_marg[mp] : 0)) return VIO_EINVAL;
        mp_to_lm[mp] = g->num_lm - 1;
    }

    if (variant == VIO_BA_LOCAL) {
        // residuals along each MapPoint's observation list, window frames only (:790-840)
        for (int mp : order) {
            for (int q = m->mp_obs_begin[mp]; q < m->mp_obs_begin[mp + 1]; ++q) {
                const int f = m->mp_obs_frame[q], fi = m->mp_obs_feat[q];
                if (f < 0 || f >= F) continue;
                if (fi < 0 || fi >= m->feat_begin[f + 1] - m->feat_begin[f]) continue;
                const int gf = m->feat_begin[f] + fi;
                if (!m->feat_valid[gf]) continue;
                if (near_boundary(m, m->feat_uv + 2 * gf)) continue;
                if (!push_obs(f, mp_to_lm[mp], gf)) return VIO_EINVAL;
            }
        }
        // NUM_FIXED_KEYFRAMES = 1: pose 0 constant when it is in the problem (:854-868)
        g->kf_const[0] = g->kf_in_problem[0];
        return VIO_OK;
    }

    // RunBA / RunVIBA: frame-major, feature order (:357-400, :567-603)
    for (int f = 0; f < F; ++f)
        for (int gf = m->feat_begin[f]; gf < m->feat_begin[f + 1]; ++gf) {
            if (!feature_usable(m, gf)) continue;
            if (near_boundary(m, m->feat_uv + 2 * gf)) continue;
            const int lm = mp_to_lm[m->feat_mp[gf]];
            if (lm < 0) continue;  // mp_to_idx.find(mp) == end
            if (!push_obs(f, lm, gf)) return VIO_EINVAL;
        }
    if (fix_first) g->kf_const[0] = 1;
    if (variant == VIO_BA_FULL && fix_last && F > 1) g->kf_const[F - 1] = 1;
    return VIO_OK;
}

extern "C" int vio_ba_write_back(const vio_map_view* m, int variant, const vio_ba_gather_out* g,
                                 const vio_ba_output* res, vio_ba_map_update* u) {
    if (!u || !g || !view_ok(m, variant)) return VIO_EINVAL;
    const int F = m->num_frames, M = m->num_mappoints;
    if (u->frame_set) std::memset(u->frame_set, 0, F);
    if (u->mp_set) std::memset(u->mp_set, 0, M);
    if (u->mp_set_bad) std::memset(u->mp_set_bad, 0, M);
    u->success = u->num_inliers = u->num_outliers = u->num_poses_optimized = u->num_points_optimized = 0;
    u->num_iterations = 0;
    u->initial_cost = u->final_cost = 0.0;
    if (g->status != VIO_GATHER_OK) return VIO_OK;  // BAResult() / PnPResult() defaults, nothing written
    if (!res || !res->summary || !res->T_wb) return VIO_EINVAL;
    const vio_ba_summary& s = *res->summary;
    u->success = s.success;
    u->num_inliers = s.num_inliers;
    u->num_outliers = s.num_outliers;
    u->initial_cost = s.initial_cost;
    u->final_cost = s.final_cost;
    u->num_iterations = s.iterations;

    if (variant == VIO_PNP) {
        // inliers < 10: keep the predicted pose (success already false in the summary); else SetTwb
        const bool accept = s.num_inliers >= 10;
        if (accept) {
            if (u->frame_set) u->frame_set[0] = 1;
            if (u->frame_Twb) pose_to_f32(&res->T_wb[0], u->frame_Twb);
        }
        return VIO_OK;
    }

    // SetBad first (the position loop below tests IsBad() afterwards)
    for (int l = 0; l < g->num_lm; ++l)
        if (res->lm_bad && res->lm_bad[l] && u->mp_set_bad) u->mp_set_bad[g->lm_mp[l]] = 1;

    u->num_points_optimized = g->num_lm;
    if (variant == VIO_BA_LOCAL) {
        for (int f = 1; f < F; ++f) {
            if (!g->kf_in_problem[f]) continue;
            if (u->frame_set) u->frame_set[f] = 1;
            if (u->frame_Twb) pose_to_f32(&res->T_wb[f], u->frame_Twb + 16 * f);
        }
        // window_frames.size() - 1 + fixed_count (:962)
        u->num_poses_optimized = F - 1 + (g->kf_in_problem[0] ? 1 : 0);
        for (int l = 0; l < g->num_lm; ++l) {
            const int mp = g->lm_mp[l];
            if (m->mp_marg[mp]) continue;
            if (u->mp_set) u->mp_set[mp] = 1;
            if (u->mp_pos && res->lm_xyz)
                for (int i = 0; i < 3; ++i) u->mp_pos[3 * mp + i] = static_cast<float>(res->lm_xyz[3 * l + i]);
        }
        return VIO_OK;
    }

    // RunBA / RunVIBA: every frame's pose (constant ones come back as SE3(T_wb_init) * exp(0))
    for (int f = 0; f < F; ++f) {
        if (u->frame_set) u->frame_set[f] = 1;
        if (u->frame_Twb) pose_to_f32(&res->T_wb[f], u->frame_Twb + 16 * f);
    }
    u->num_poses_optimized = F;
    if (variant == VIO_BA_VI) {
        if (u->frame_vel && res->vel)
            for (int i = 0; i < 3 * F; ++i) u->frame_vel[i] = static_cast<float>(res->vel[i]);
        if (u->bias && res->bg && res->ba)
            for (int i = 0; i < 3; ++i) {
                u->bias[i] = static_cast<float>(res->bg[i]);
                u->bias[3 + i] = static_cast<float>(res->ba[i]);
            }
    }
    for (int l = 0; l < g->num_lm; ++l) {
        const int mp = g->lm_mp[l];
        const bool bad = res->lm_bad && res->lm_bad[l];
        if (bad || m->mp_marg[mp]) continue;
        if (u->mp_set) u->mp_set[mp] = 1;
        if (u->mp_pos && res->lm_xyz)
            for (int i = 0; i < 3; ++i) u->mp_pos[3 * mp + i] = static_cast<float>(res->lm_xyz[3 * l + i]);
    }
    return VIO_OK;
}
