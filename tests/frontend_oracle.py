"""TEST INFRASTRUCTURE: restatement of FeatureTracker::TrackFeatures' host bookkeeping
(src/processing/FeatureTracker.cpp:61-206, :404-497; src/database/Frame.cpp:108-202) on top of the
C oracle's numeric functions (oracle_lib).  Used only by tests/test_frontend_gpu.py."""
import numpy as np

import oracle_lib


def libstdcxx_sort_small(idx, key):
    """std::sort(begin, end, [](a, b){ return key(a) > key(b); }) for n <= 16: libstdc++ skips the
    introsort loop (threshold 16) and runs __insertion_sort, which keeps equal keys in order."""
    assert len(idx) <= 16, "cell larger than libstdc++'s insertion-sort threshold"
    out = list(idx)
    for i in range(1, len(out)):
        v = out[i]
        j = i
        while j > 0 and key(v) > key(out[j - 1]):
            out[j] = out[j - 1]
            j -= 1
        out[j] = v
    return out


def assign_and_limit(feats, W, H, gc, gr, max_per):
    cw, ch = np.float32(W) / np.float32(gc), np.float32(H) / np.float32(gr)
    grid = [[] for _ in range(gc * gr)]
    for i, f in enumerate(feats):
        x, y = f["x"], f["y"]
        if x < 0 or x >= W or y < 0 or y >= H:
            continue
        gx = min(int(np.float32(x) / cw), gc - 1)
        gy = min(int(np.float32(y) / ch), gr - 1)
        grid[gy * gc + gx].append(i)
    keep = set()
    for cell in grid:
        if len(cell) > max_per:
            cell = libstdcxx_sort_small(cell, lambda i: feats[i]["tc"])[:max_per]
        keep.update(cell)
    return [f for i, f in enumerate(feats) if i in keep]


def remove_clustered(feats, W, H, ratio):
    if len(feats) < 4:
        return feats
    gc, gr = 20, 10
    cw, ch = np.float32(W) / np.float32(gc), np.float32(H) / np.float32(gr)
    thr = np.float32(np.sqrt(np.float32(cw * cw + ch * ch))) * np.float32(ratio)

    def cell_of(f):
        return min(int(np.float32(f["y"]) / ch), gr - 1) * gc + min(int(np.float32(f["x"]) / cw), gc - 1)

    cells = {}
    for i, f in enumerate(feats):
        cells.setdefault(cell_of(f), []).append(i)
    clustered = set()
    for c, idx in cells.items():
        if len(idx) < 4:
            continue
        mx, my = np.float32(0), np.float32(0)
        for i in idx:
            mx = np.float32(mx + np.float32(feats[i]["x"]))
            my = np.float32(my + np.float32(feats[i]["y"]))
        mx = np.float32(mx / np.float32(len(idx)))
        my = np.float32(my / np.float32(len(idx)))
        var = np.float32(0)
        for i in idx:
            dx = np.float32(np.float32(feats[i]["x"]) - mx)
            dy = np.float32(np.float32(feats[i]["y"]) - my)
            var = np.float32(var + np.float32(dx * dx + dy * dy))
        var = np.float32(var / np.float32(len(idx)))
        if np.sqrt(var) < thr:
            clustered.add(c)
    return [f for f in feats if cell_of(f) not in clustered]


def cv_circle_fill(mask, cx, cy, r):
    h, w = mask.shape
    err, dx, dy, plus, minus = 0, r, 0, 1, (r << 1) - 1
    while dx >= dy:
        for (yy, xl, xr) in ((cy - dy, cx - dx, cx + dx), (cy + dy, cx - dx, cx + dx),
                             (cy - dx, cx - dy, cx + dy), (cy + dx, cx - dy, cx + dy)):
            if 0 <= yy < h:
                mask[yy, max(xl, 0):min(xr, w - 1) + 1] = 0
        dy += 1
        err += plus
        plus += 2
        m = (err <= 0) - 1
        err -= minus & m
        dx += m
        minus -= m & 2


class FrontendOracle:
    def __init__(self, vio, W, H, params):
        self.vio, self.W, self.H, self.p = vio, W, H, params
        self.feats = []
        self.next_id = 0
        self.frame = 0
        self.prev = None

    def _base_mask(self):
        W, H = self.W, self.H
        m = np.zeros((H, W), np.uint8)
        m[int(np.float32(H) * np.float32(0.15)):int(np.float32(H) * (np.float32(1.0) - np.float32(0.15))),
          self.p.boundary_margin:W - self.p.boundary_margin] = 255
        return m

    def _detect(self, img, with_discs):
        m = self._base_mask()
        if with_discs:
            r = int(self.p.min_distance)
            for f in self.feats:
                cv_circle_fill(m, int(np.rint(np.float32(f["x"]))), int(np.rint(np.float32(f["y"]))), r)
        return oracle_lib.gftt(img, m, self.p.max_features, float(np.float32(self.p.quality_level)),
                               float(np.float32(self.p.min_distance)))

    def track(self, img):
        p, W, H = self.p, self.W, self.H
        if self.frame == 0 or not self.feats:
            c = self._detect(img, False)
            self.feats = [dict(id=self.next_id + i, x=float(x), y=float(y), tc=0, age=0) for i, (x, y) in enumerate(c)]
            self.next_id += len(c)
            self.num_tracked, self.num_detected = 0, len(c)
            self.feats = assign_and_limit(self.feats, W, H, p.grid_cols, p.grid_rows, p.max_features_per_grid)
        else:
            prev = np.array([[f["x"], f["y"]] for f in self.feats], np.float32)
            nxt, st, _ = oracle_lib.klt_track(self.prev, img, prev, self.vio.default_klt_params())
            m = np.float32(p.boundary_margin)
            good = []
            for i in range(len(prev)):
                x, y = nxt[i]
                vr = np.float32(y / np.float32(H))
                polar = vr < np.float32(0.15) or vr > np.float32(1.0) - np.float32(0.15)
                nearb = x < m or x > np.float32(W) - m or y < m or y > np.float32(H) - m
                if st[i] and not polar and not nearb:
                    good.append(i)
            inl = np.ones(len(good), np.uint8)
            if len(good) >= 3:
                s = self.vio.ransac_samples((p.ransac_seed + self.frame) & 0xffffffff, len(good), 1000)
                inl, _ = oracle_lib.rot_ransac(prev[good], nxt[good], W, H, s, self.vio.ransac_threshold())
            cur = []
            for j, i in enumerate(good):
                if inl[j]:
                    f = self.feats[i]
                    cur.append(dict(id=f["id"], x=float(nxt[i, 0]), y=float(nxt[i, 1]), tc=f["tc"] + 1, age=f["age"] + 1))
            self.feats = cur
            self.num_tracked = len(cur)
            if p.remove_clustered:
                self.feats = remove_clustered(self.feats, W, H, p.clustered_std_ratio)
            self.feats = assign_and_limit(self.feats, W, H, p.grid_cols, p.grid_rows, p.max_features_per_grid)
            if len(self.feats) < p.max_features:
                c = self._detect(img, True)
                self.feats += [dict(id=self.next_id + i, x=float(x), y=float(y), tc=0, age=0) for i, (x, y) in enumerate(c)]
                self.next_id += len(c)
                self.num_detected = len(c)
                self.feats = assign_and_limit(self.feats, W, H, p.grid_cols, p.grid_rows, p.max_features_per_grid)
            else:
                self.num_detected = 0
        self.prev = img
        self.frame += 1
        return {"ids": np.array([f["id"] for f in self.feats], np.int32),
                "xy": np.array([[f["x"], f["y"]] for f in self.feats], np.float32).reshape(-1, 2),
                "track_count": np.array([f["tc"] for f in self.feats], np.int32),
                "age": np.array([f["age"] for f in self.feats], np.int32),
                "num_tracked": self.num_tracked, "num_detected": self.num_detected}
