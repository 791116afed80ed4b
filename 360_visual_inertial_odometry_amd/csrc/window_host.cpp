// window_host.cpp — the Estimator's sliding-window bookkeeping on a host-side graph.
//
// Reference (src/processing/Estimator.cpp, src/database/MapPoint.cpp, Frame.cpp):
//   CreateKeyframe            :671-754   keyframe appended; observations of its linked MapPoints added
//                                        (MapPoint::AddObservation updates an existing frame's index in
//                                        place); while the window exceeds max_keyframes the oldest
//                                        keyframe leaves: MapPoints it references move their reference
//                                        to the oldest in-window keyframe observing them and become
//                                        marginalised, or are set bad; then its observations are
//                                        removed (MapPoint::RemoveObservation: bad when none remain).
//   LinkMapPointsFromPreviousFrame :806-843
//   TriangulateNewMapPoints   :1141-1318 feature-id matching (unordered_map: the last valid kf1 feature
//                                        of an id wins), kf2 features with a good MapPoint skipped,
//                                        TriangulateSinglePoint (device: vio_triangulate), new MapPoint
//                                        with reference kf1 and observations kf1, kf2 and the in-window
//                                        keyframes of kf2's feature track (the pixel-error gate is
//                                        commented out in the reference: every valid point is kept).
// The IMU preintegration of :646-666 is the caller's (vio_imu_preintegrate), the BA that follows
// (:763-798) is vio_ba_gather / vio_ba_solve / vio_ba_write_back over vio_window_map_view.
// Frames never expire here (the reference's weak_ptr observations of destroyed frames are dropped by
// RemoveObservation; keyframes stay alive in m_all_keyframes).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <deque>
#include <unordered_map>
#include <vector>

#include "vio360.h"

namespace {

struct WFrame {
    int32_t id = 0, width = 0;
    float Twb[16], Tbc[16];
    std::vector<int32_t> fid, mp;
    std::vector<float> uv, bearing;
    std::vector<uint8_t> valid;
    std::vector<int32_t> tbeg, tframe, tfeat;  // feature tracks (CSR)
};

struct WMap {
    float pos[3];
    bool bad = false, marg = false, tri = false;
    int32_t ref = -1;
    std::vector<std::pair<int32_t, int32_t>> obs;  // (frame id, feature index), insertion order
};

void mul4(const float* A, const float* B, float* C) {
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c)
            C[4 * r + c] = ((A[4 * r] * B[c] + A[4 * r + 1] * B[4 + c]) + A[4 * r + 2] * B[8 + c]) + A[4 * r + 3] * B[12 + c];
}
// inverse of a rigid 4x4 transform (the reference inverts the general matrix; these are rigid)
void rigid_inv(const float* T, float* Ti) {
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) Ti[4 * r + c] = T[4 * c + r];
        Ti[4 * r + 3] = -((T[r] * T[3] + T[4 + r] * T[7]) + T[8 + r] * T[11]);
    }
    Ti[12] = Ti[13] = Ti[14] = 0.f;
    Ti[15] = 1.f;
}

}  // namespace

struct vio_window {
    int max_kf = 10;
    std::vector<WFrame> frames;                 // every keyframe ever added (m_all_keyframes)
    std::unordered_map<int32_t, int> by_id;      // frame id -> index in frames
    std::deque<int> win;                         // m_keyframes: indices into frames, oldest first
    std::vector<WMap> mps;
    // map-view staging (vio_window_map_view)
    std::vector<int> view_frames;
    std::vector<float> v_twb, v_tcb, v_uv, v_pos;
    std::vector<int32_t> v_fbeg, v_fmp, v_obeg, v_oframe, v_ofeat;
    std::vector<uint8_t> v_valid, v_bad, v_marg;
    std::vector<int64_t> v_key;

    WFrame* frame(int32_t id) {
        auto it = by_id.find(id);
        return it == by_id.end() ? nullptr : &frames[it->second];
    }
    const WFrame* frame(int32_t id) const {
        auto it = by_id.find(id);
        return it == by_id.end() ? nullptr : &frames[it->second];
    }
    bool in_window(int32_t id) const {
        for (int f : win)
            if (frames[f].id == id) return true;
        return false;
    }
    bool observed_by(const WMap& m, int32_t id) const {
        for (const auto& o : m.obs)
            if (o.first == id) return true;
        return false;
    }
    void add_obs(WMap& m, int32_t id, int32_t feat) {  // MapPoint::AddObservation
        for (auto& o : m.obs)
            if (o.first == id) {
                o.second = feat;
                return;
            }
        m.obs.emplace_back(id, feat);
    }
    void remove_obs(WMap& m, int32_t id) {  // MapPoint::RemoveObservation
        m.obs.erase(std::remove_if(m.obs.begin(), m.obs.end(), [&](const std::pair<int32_t, int32_t>& o) { return o.first == id; }),
                    m.obs.end());
        if (m.obs.empty()) m.bad = true;
    }
    bool good(int32_t h) const { return h >= 0 && h < (int32_t)mps.size() && !mps[h].bad; }
};

extern "C" {

int vio_window_create(int max_keyframes, vio_window** out) {
    if (!out || max_keyframes < 1) return VIO_EINVAL;
    *out = new vio_window();
    (*out)->max_kf = max_keyframes;
    return VIO_OK;
}

void vio_window_destroy(vio_window* win) { delete win; }

int vio_window_add_mappoint(vio_window* win, const float* pos, int32_t reference_frame, int32_t* handle) {
    if (!win || !pos || !handle) return VIO_EINVAL;
    WMap m;
    std::memcpy(m.pos, pos, sizeof(m.pos));
    m.ref = reference_frame;
    win->mps.push_back(m);
    *handle = (int32_t)win->mps.size() - 1;
    return VIO_OK;
}

int vio_window_add_observation(vio_window* win, int32_t mp, int32_t frame_id, int32_t feat) {
    if (!win || mp < 0 || mp >= (int32_t)win->mps.size()) return VIO_EINVAL;
    WFrame* f = win->frame(frame_id);
    if (!f || feat < 0 || feat >= (int32_t)f->fid.size()) return VIO_EINVAL;
    win->add_obs(win->mps[mp], frame_id, feat);
    f->mp[feat] = mp;
    return VIO_OK;
}

int vio_window_link_mappoints(const vio_window* win, const int32_t* prev_id, const uint8_t* prev_valid,
                              const int32_t* prev_mp, int n_prev, const int32_t* curr_id, int n_curr, int32_t* curr_mp) {
    if (!win || n_prev < 0 || n_curr < 0 || (n_prev > 0 && (!prev_id || !prev_valid || !prev_mp)) ||
        (n_curr > 0 && (!curr_id || !curr_mp)))
        return VIO_EINVAL;
    std::unordered_map<int32_t, int> prev;
    for (int i = 0; i < n_prev; ++i)
        if (prev_valid[i]) prev[prev_id[i]] = i;
    for (int i = 0; i < n_curr; ++i) {
        curr_mp[i] = -1;
        auto it = prev.find(curr_id[i]);
        if (it != prev.end() && win->good(prev_mp[it->second])) curr_mp[i] = prev_mp[it->second];
    }
    return VIO_OK;
}

int vio_window_add_keyframe(vio_window* win, const vio_window_frame* fr, vio_window_kf_stats* stats) {
    if (!win || !fr || fr->num_features < 0 || !fr->T_wb || !fr->T_bc || win->by_id.count(fr->frame_id)) return VIO_EINVAL;
    const int n = fr->num_features;
    if (n > 0 && (!fr->feature_id || !fr->bearing || !fr->valid || !fr->mappoint)) return VIO_EINVAL;
    for (int i = 0; i < n; ++i)
        if (fr->mappoint[i] < -1 || fr->mappoint[i] >= (int32_t)win->mps.size()) return VIO_EINVAL;
    WFrame f;
    f.id = fr->frame_id;
    f.width = fr->width;
    std::memcpy(f.Twb, fr->T_wb, sizeof(f.Twb));
    std::memcpy(f.Tbc, fr->T_bc, sizeof(f.Tbc));
    f.fid.assign(fr->feature_id, fr->feature_id + n);
    f.mp.assign(fr->mappoint, fr->mappoint + n);
    f.valid.assign(fr->valid, fr->valid + n);
    f.bearing.assign(fr->bearing, fr->bearing + 3 * n);
    if (fr->uv) f.uv.assign(fr->uv, fr->uv + 2 * n);
    else f.uv.assign(2 * (size_t)n, 0.f);
    f.tbeg.assign(n + 1, 0);
    if (fr->track_begin && n > 0) {
        f.tbeg.assign(fr->track_begin, fr->track_begin + n + 1);
        const int nt = f.tbeg[n] - f.tbeg[0];
        if (nt < 0 || f.tbeg[0] < 0 || !fr->track_frame || !fr->track_feat) return VIO_EINVAL;
        for (int i = 0; i < n; ++i)  // CSR offsets: monotonic, so every feature's range lies in [0, nt)
            if (f.tbeg[i] > f.tbeg[i + 1]) return VIO_EINVAL;
        for (int i = 0; i <= n; ++i) f.tbeg[i] -= fr->track_begin[0];
        f.tframe.assign(fr->track_frame + fr->track_begin[0], fr->track_frame + fr->track_begin[0] + nt);
        f.tfeat.assign(fr->track_feat + fr->track_begin[0], fr->track_feat + fr->track_begin[0] + nt);
    }
    vio_window_kf_stats st{};
    st.removed_frame = -1;
    win->frames.push_back(std::move(f));
    const int fi = (int)win->frames.size() - 1;
    win->by_id[fr->frame_id] = fi;
    win->win.push_back(fi);
    // :679-690
    {
        WFrame& cur = win->frames[fi];
        for (int i = 0; i < n; ++i) {
            const int32_t h = cur.mp[i];
            if (win->good(h) && cur.valid[i] && !win->observed_by(win->mps[h], cur.id)) {
                win->add_obs(win->mps[h], cur.id, i);
                st.obs_added++;
            }
        }
    }
    // :693-754
    while ((int)win->win.size() > win->max_kf) {
        const WFrame& old = win->frames[win->win.front()];
        for (size_t i = 0; i < old.mp.size(); ++i) {
            const int32_t h = old.mp[i];
            if (!win->good(h)) continue;
            WMap& m = win->mps[h];
            if (m.ref != old.id) continue;
            int32_t nref = -1;
            for (size_t k = 1; k < win->win.size(); ++k) {
                const int32_t kid = win->frames[win->win[k]].id;
                if (win->observed_by(m, kid)) {
                    nref = kid;
                    break;
                }
            }
            if (nref >= 0) {
                m.ref = nref;
                m.marg = true;
                st.transferred++;
            } else {
                m.bad = true;
                st.deleted++;
            }
        }
        for (size_t i = 0; i < old.mp.size(); ++i) {
            const int32_t h = old.mp[i];
            if (!win->good(h)) continue;
            win->remove_obs(win->mps[h], old.id);
        }
        st.removed_frame = old.id;
        win->win.pop_front();
    }
    st.num_keyframes = (int)win->win.size();
    if (stats) *stats = st;
    return VIO_OK;
}

int vio_window_triangulation_candidates(const vio_window* win, int32_t kf1_id, int32_t kf2_id, int32_t* pairs,
                                        float* bearings, float* T_cw, int cap, int* n) {
    if (!win || !n || cap < 0) return VIO_EINVAL;
    const WFrame* a = win->frame(kf1_id);
    const WFrame* b = win->frame(kf2_id);
    if (!a || !b) return VIO_EINVAL;
    std::unordered_map<int32_t, int> m1;  // :1157-1162
    for (size_t i = 0; i < a->fid.size(); ++i)
        if (a->valid[i]) m1[a->fid[i]] = (int)i;
    int c = 0;
    for (size_t i2 = 0; i2 < b->fid.size(); ++i2) {  // :1190-1221
        if (!b->valid[i2]) continue;
        auto it = m1.find(b->fid[i2]);
        if (it == m1.end()) continue;
        if (win->good(b->mp[i2])) continue;
        if (c < cap && pairs && bearings) {
            const int i1 = it->second;
            pairs[2 * c] = i1;
            pairs[2 * c + 1] = (int32_t)i2;
            for (int k = 0; k < 3; ++k) {
                bearings[6 * c + k] = a->bearing[3 * i1 + k];
                bearings[6 * c + 3 + k] = b->bearing[3 * i2 + k];
            }
        }
        ++c;
    }
    if (T_cw) {  // GetTwc().inverse() = (T_wb T_bc)^-1
        float Twc[16];
        mul4(a->Twb, a->Tbc, Twc);
        rigid_inv(Twc, T_cw);
        mul4(b->Twb, b->Tbc, Twc);
        rigid_inv(Twc, T_cw + 16);
    }
    *n = c;
    return VIO_OK;
}

int vio_window_commit_triangulation(vio_window* win, int32_t kf1_id, int32_t kf2_id, const int32_t* pairs,
                                    const float* points, const uint8_t* valid, int n, int32_t* new_mp, int* n_new) {
    if (!win || n < 0 || (n > 0 && (!pairs || !points || !valid))) return VIO_EINVAL;
    WFrame* a = win->frame(kf1_id);
    WFrame* b = win->frame(kf2_id);
    if (!a || !b) return VIO_EINVAL;
    for (int c = 0; c < n; ++c)
        if (pairs[2 * c] < 0 || pairs[2 * c] >= (int32_t)a->fid.size() || pairs[2 * c + 1] < 0 ||
            pairs[2 * c + 1] >= (int32_t)b->fid.size())
            return VIO_EINVAL;
    int made = 0;
    for (int c = 0; c < n; ++c) {
        if (new_mp) new_mp[c] = -1;
        if (!valid[c]) continue;  // depth_failed (:1218-1221)
        const int i1 = pairs[2 * c], i2 = pairs[2 * c + 1];
        WMap m;
        std::memcpy(m.pos, points + 3 * c, sizeof(m.pos));
        m.tri = true;
        m.ref = a->id;
        win->mps.push_back(m);
        const int32_t h = (int32_t)win->mps.size() - 1;
        // frames may be re-fetched: mps grew, frames did not
        win->add_obs(win->mps[h], a->id, i1);
        win->add_obs(win->mps[h], b->id, i2);
        a->mp[i1] = h;
        b->mp[i2] = h;
        // :1269-1309: in-window keyframes of kf2's feature track
        for (int t = b->tbeg[i2]; t < b->tbeg[i2 + 1]; ++t) {
            const int32_t oid = b->tframe[t];
            if (oid == a->id || oid == b->id) continue;
            WFrame* of = win->frame(oid);
            if (!of || !win->in_window(oid)) continue;  // IsKeyframe / IsKeyframeInWindow
            const int32_t idx = b->tfeat[t];
            if (idx < 0 || idx >= (int32_t)of->fid.size()) continue;
            win->add_obs(win->mps[h], oid, idx);
            of->mp[idx] = h;
        }
        if (new_mp) new_mp[c] = h;
        ++made;
    }
    if (n_new) *n_new = made;
    return VIO_OK;
}

int vio_window_triangulate(vio_window* win, vio_ctx* ctx, int32_t kf1_id, int32_t kf2_id, int* n_new) {
    if (!win || !ctx) return VIO_EINVAL;
    int n = 0;
    int rc = vio_window_triangulation_candidates(win, kf1_id, kf2_id, nullptr, nullptr, nullptr, 0, &n);
    if (rc) return rc;
    std::vector<int32_t> pairs(2 * (size_t)n), pp(2 * (size_t)n);
    std::vector<float> bear(6 * (size_t)n), T(32), X(3 * (size_t)n);
    std::vector<uint8_t> valid(n);
    rc = vio_window_triangulation_candidates(win, kf1_id, kf2_id, pairs.data(), bear.data(), T.data(), n, &n);
    if (rc) return rc;
    if (n > 0) {
        for (int c = 0; c < n; ++c) {
            pp[2 * c] = 0;
            pp[2 * c + 1] = 1;
        }
        rc = vio_triangulate(ctx, T.data(), 2, pp.data(), bear.data(), n, win->frame(kf1_id)->width, X.data(),
                             valid.data(), nullptr);
        if (rc) return rc;
    }
    return vio_window_commit_triangulation(win, kf1_id, kf2_id, pairs.data(), X.data(), valid.data(), n, nullptr, n_new);
}

int vio_window_keyframes(const vio_window* win, int32_t* frame_ids, int cap, int* n) {
    if (!win || !n || cap < 0) return VIO_EINVAL;
    int k = 0;
    for (int f : win->win) {
        if (k < cap && frame_ids) frame_ids[k] = win->frames[f].id;
        ++k;
    }
    *n = k;
    return VIO_OK;
}

int vio_window_num_mappoints(const vio_window* win) { return win ? (int)win->mps.size() : VIO_EINVAL; }

int vio_window_mappoint(const vio_window* win, int32_t mp, vio_window_mappoint_info* info) {
    if (!win || !info || mp < 0 || mp >= (int32_t)win->mps.size()) return VIO_EINVAL;
    const WMap& m = win->mps[mp];
    std::memcpy(info->pos, m.pos, sizeof(m.pos));
    info->bad = m.bad;
    info->marginalized = m.marg;
    info->triangulated = m.tri;
    info->reference_frame = m.ref;
    info->num_observations = (int32_t)m.obs.size();
    return VIO_OK;
}

int vio_window_mappoint_observations(const vio_window* win, int32_t mp, int32_t* frame_ids, int32_t* feats, int cap,
                                     int* n) {
    if (!win || !n || cap < 0 || mp < 0 || mp >= (int32_t)win->mps.size()) return VIO_EINVAL;
    const WMap& m = win->mps[mp];
    for (int k = 0; k < (int)m.obs.size() && k < cap; ++k) {
        if (frame_ids) frame_ids[k] = m.obs[k].first;
        if (feats) feats[k] = m.obs[k].second;
    }
    *n = (int)m.obs.size();
    return VIO_OK;
}

int vio_window_frame_mappoints(const vio_window* win, int32_t frame_id, int32_t* mp, int cap, int* n) {
    if (!win || !n || cap < 0) return VIO_EINVAL;
    const WFrame* f = win->frame(frame_id);
    if (!f) return VIO_EINVAL;
    for (int k = 0; k < (int)f->mp.size() && k < cap; ++k)
        if (mp) mp[k] = f->mp[k];
    *n = (int)f->mp.size();
    return VIO_OK;
}

int vio_window_map_view(vio_window* w, int height, int boundary_margin, vio_map_view* v) {
    if (!w || !v) return VIO_EINVAL;
    w->view_frames.assign(w->win.begin(), w->win.end());
    const int F = (int)w->view_frames.size(), M = (int)w->mps.size();
    w->v_twb.resize(16 * (size_t)F);
    w->v_tcb.resize(16 * (size_t)F);
    w->v_fbeg.assign(1, 0);
    w->v_uv.clear();
    w->v_valid.clear();
    w->v_fmp.clear();
    std::unordered_map<int32_t, int> slot;
    for (int s = 0; s < F; ++s) {
        const WFrame& f = w->frames[w->view_frames[s]];
        slot[f.id] = s;
        std::memcpy(&w->v_twb[16 * s], f.Twb, sizeof(f.Twb));
        rigid_inv(f.Tbc, &w->v_tcb[16 * s]);  // GetTCB() = T_BC^-1
        w->v_uv.insert(w->v_uv.end(), f.uv.begin(), f.uv.end());
        w->v_valid.insert(w->v_valid.end(), f.valid.begin(), f.valid.end());
        w->v_fmp.insert(w->v_fmp.end(), f.mp.begin(), f.mp.end());
        w->v_fbeg.push_back((int32_t)w->v_fmp.size());
    }
    w->v_key.resize(M);
    w->v_bad.resize(M);
    w->v_marg.resize(M);
    w->v_pos.resize(3 * (size_t)M);
    w->v_obeg.assign(1, 0);
    w->v_oframe.clear();
    w->v_ofeat.clear();
    for (int m = 0; m < M; ++m) {
        const WMap& p = w->mps[m];
        w->v_key[m] = m;
        w->v_bad[m] = p.bad;
        w->v_marg[m] = p.marg;
        std::memcpy(&w->v_pos[3 * m], p.pos, sizeof(p.pos));
        for (const auto& o : p.obs) {
            auto it = slot.find(o.first);
            w->v_oframe.push_back(it == slot.end() ? -1 : it->second);
            w->v_ofeat.push_back(o.second);
        }
        w->v_obeg.push_back((int32_t)w->v_oframe.size());
    }
    std::memset(v, 0, sizeof(*v));
    v->num_frames = F;
    v->num_mappoints = M;
    v->frame_Twb = w->v_twb.data();
    v->frame_Tcb = w->v_tcb.data();
    v->feat_begin = w->v_fbeg.data();
    v->feat_uv = w->v_uv.data();
    v->feat_valid = w->v_valid.data();
    v->feat_mp = w->v_fmp.data();
    v->mp_key = w->v_key.data();
    v->mp_bad = w->v_bad.data();
    v->mp_marg = w->v_marg.data();
    v->mp_pos = w->v_pos.data();
    v->mp_obs_begin = w->v_obeg.data();
    v->mp_obs_frame = w->v_oframe.data();
    v->mp_obs_feat = w->v_ofeat.data();
    v->width = F ? w->frames[w->view_frames[0]].width : 0;
    v->height = height;
    v->boundary_margin = boundary_margin;
    return VIO_OK;
}

int vio_window_apply_update(vio_window* w, const vio_ba_map_update* u) {
    if (!w || !u) return VIO_EINVAL;
    const int F = (int)w->view_frames.size(), M = (int)w->v_key.size();
    if (M > (int)w->mps.size()) return VIO_EINVAL;
    for (int s = 0; s < F; ++s)
        if (u->frame_set && u->frame_Twb && u->frame_set[s])
            std::memcpy(w->frames[w->view_frames[s]].Twb, u->frame_Twb + 16 * s, sizeof(float) * 16);
    for (int m = 0; m < M; ++m) {
        if (u->mp_set_bad && u->mp_set_bad[m]) w->mps[m].bad = true;
        if (u->mp_set && u->mp_pos && u->mp_set[m]) std::memcpy(w->mps[m].pos, u->mp_pos + 3 * m, sizeof(float) * 3);
    }
    return VIO_OK;
}

}  // extern "C"
