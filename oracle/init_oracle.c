/* init_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker / CPU baseline), never a product path.
 *
 * CPU restatement of Initializer::TryMonocularInitialization's numeric core
 * (src/processing/Initializer.cpp:47-291 of the reference):
 *   ComputeEssentialMatrix  :458-621   8-point RANSAC (samples injected: the reference seeds mt19937
 *                                      from std::random_device, :477-480), |b2^T E b1| < thr inliers,
 *                                      first strictly-best hypothesis, refit on its inliers;
 *   RecoverPose             :623-697   candidates (R1, t1), (R1, -t1), (R2, t1), (R2, -t1);
 *   TestPoseCandidate       :785-835   mid-point triangulation + reprojection < 5 px in both frames;
 *   TriangulatePoints       :699-726,  TriangulateSinglePoint :728-783;
 *   ValidateInitialization  :889-995,  ComputeReprojectionErrorInFrame :837-871;
 *   NormalizeScale          :997-1048.
 * The reference solves the null vectors / SVDs with Eigen's f32 JacobiSVD (Eigen is absent from the
 * image: parity with it is unpinned).  This restatement — like the device path — takes the null
 * vector as the smallest-eigenvalue eigenvector of G = A^T A in f64 (cyclic Jacobi), with a fixed
 * sign, and the 3x3 SVDs through the eigen-decomposition of M^T M; the refit's sum over inliers is
 * restated in the fixed order the device uses (64 strided partial sums, then in lane order).  The
 * per-point f32 expressions are the reference's.  Pinned by closed forms in tests/test_init_oracle.py
 * (noise-free two-view geometry: E = [t]x R up to scale, exact R / t direction, zero epipolar
 * residuals, the four-candidate set).  Compile with -ffp-contract=off.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int32_t width, height, min_features, ransac_iterations;
    float ransac_threshold, max_reprojection_error;
} oi_params;

typedef struct {
    int32_t status, best_hypothesis, num_inliers, pose_candidate;
    int32_t candidate_good[4];
    int32_t num_triangulated, num_valid;
    float mean_reproj_error, scale_factor;
    float E[9], R[9], t[3];
} oi_result;

static void epi_row(const float* b1, const float* b2, float* row) {
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) row[3 * r + c] = b2[r] * b1[c];
}

static float epi_err(const float* E, const float* b1, const float* b2) {
    float w[3];
    for (int c = 0; c < 3; ++c) w[c] = (b2[0] * E[c] + b2[1] * E[3 + c]) + b2[2] * E[6 + c];
    return fabsf((w[0] * b1[0] + w[1] * b1[1]) + w[2] * b1[2]);
}

/* cyclic Jacobi on a symmetric n x n row-major matrix; V <- eigenvectors (columns) */
static void jacobi(double* A, double* V, int n) {
    for (int p = 0; p < n; ++p)
        for (int q = 0; q < n; ++q) V[p * n + q] = p == q ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 50; ++sweep) {
        double off = 0.0, dg = 0.0;
        for (int p = 0; p < n; ++p) {
            dg += A[p * n + p] * A[p * n + p];
            for (int q = p + 1; q < n; ++q) off += A[p * n + q] * A[p * n + q];
        }
        if (!(off > 1e-32 * dg)) break;
        for (int p = 0; p < n - 1; ++p)
            for (int q = p + 1; q < n; ++q) {
                const double apq = A[p * n + q];
                if (apq == 0.0) continue;
                const double app = A[p * n + p], aqq = A[q * n + q];
                const double theta = (aqq - app) / (2.0 * apq);
                const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < n; ++k) {
                    if (k == p || k == q) continue;
                    const double akp = A[k * n + p], akq = A[k * n + q];
                    const double np = c * akp - s * akq, nq = s * akp + c * akq;
                    A[k * n + p] = A[p * n + k] = np;
                    A[k * n + q] = A[q * n + k] = nq;
                }
                A[p * n + p] = app - t * apq;
                A[q * n + q] = aqq + t * apq;
                A[p * n + q] = A[q * n + p] = 0.0;
                for (int k = 0; k < n; ++k) {
                    const double vkp = V[k * n + p], vkq = V[k * n + q];
                    V[k * n + p] = c * vkp - s * vkq;
                    V[k * n + q] = s * vkp + c * vkq;
                }
            }
    }
}

static void null_vector9(double* G, double* e) {
    double V[81];
    jacobi(G, V, 9);
    int kmin = 0;
    for (int k = 1; k < 9; ++k)
        if (G[k * 9 + k] < G[kmin * 9 + kmin]) kmin = k;
    int imax = 0;
    for (int i = 0; i < 9; ++i) {
        e[i] = V[i * 9 + kmin];
        if (fabs(e[i]) > fabs(e[imax])) imax = i;
    }
    if (e[imax] < 0.0)
        for (int i = 0; i < 9; ++i) e[i] = -e[i];
}

/* SVD of a 3x3 f32 matrix via eig(M^T M) in f64: s descending, u[k] = M v[k] / s[k] (k < 2),
   u2 = u0 x u1, v2 = v0 x v1 */
static void svd3(const float* M, double u[3][3], double* s, double v[3][3]) {
    double A[9], V[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            A[3 * i + j] = ((double)M[i] * (double)M[j] + (double)M[3 + i] * (double)M[3 + j]) +
                           (double)M[6 + i] * (double)M[6 + j];
    jacobi(A, V, 3);
    int o[3] = {0, 1, 2};
    for (int i = 1; i < 3; ++i)
        for (int j = i; j > 0 && A[4 * o[j]] > A[4 * o[j - 1]]; --j) {
            int tmp = o[j];
            o[j] = o[j - 1];
            o[j - 1] = tmp;
        }
    for (int k = 0; k < 3; ++k) {
        const double l = A[4 * o[k]];
        s[k] = l > 0.0 ? sqrt(l) : 0.0;
        for (int i = 0; i < 3; ++i) v[k][i] = V[3 * i + o[k]];
    }
    for (int k = 0; k < 2; ++k)
        for (int i = 0; i < 3; ++i) {
            const double mv = ((double)M[3 * i] * v[k][0] + (double)M[3 * i + 1] * v[k][1]) + (double)M[3 * i + 2] * v[k][2];
            u[k][i] = s[k] > 0.0 ? mv / s[k] : 0.0;
        }
    u[2][0] = u[0][1] * u[1][2] - u[0][2] * u[1][1];
    u[2][1] = u[0][2] * u[1][0] - u[0][0] * u[1][2];
    u[2][2] = u[0][0] * u[1][1] - u[0][1] * u[1][0];
    v[2][0] = v[0][1] * v[1][2] - v[0][2] * v[1][1];
    v[2][1] = v[0][2] * v[1][0] - v[0][0] * v[1][2];
    v[2][2] = v[0][0] * v[1][1] - v[0][1] * v[1][0];
}

/* :525-538 / :611-616: E <- U diag(s, s, 0) V^T with s = (s0 + s1) / 2 */
static void project_essential(const double* e, float* E) {
    float Ec[9];
    double u[3][3], s[3], v[3][3];
    for (int k = 0; k < 9; ++k) Ec[k] = (float)e[k];
    svd3(Ec, u, s, v);
    const double sigma = (s[0] + s[1]) * 0.5;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) E[3 * i + j] = (float)(sigma * (u[0][i] * v[0][j] + u[1][i] * v[1][j]));
}

static float det3f(const float* m) {
    return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) + m[2] * (m[3] * m[7] - m[4] * m[6]);
}

/* :636-663 */
static void pose_candidates(const float* E, float Rc[4][9], float tc[4][3]) {
    double u[3][3], s[3], v[3][3];
    float R1[9], R2[9], t1[3];
    svd3(E, u, s, v);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            R1[3 * i + j] = (float)((u[1][i] * v[0][j] - u[0][i] * v[1][j]) + u[2][i] * v[2][j]); /* U W V^T */
            R2[3 * i + j] = (float)((u[0][i] * v[1][j] - u[1][i] * v[0][j]) + u[2][i] * v[2][j]); /* U W^T V^T */
        }
    for (int k = 0; k < 3; ++k) t1[k] = (float)u[2][k];
    if (det3f(R1) < 0.f) {
        for (int k = 0; k < 9; ++k) R1[k] = -R1[k];
        for (int k = 0; k < 3; ++k) t1[k] = -t1[k];
    }
    if (det3f(R2) < 0.f)
        for (int k = 0; k < 9; ++k) R2[k] = -R2[k];
    const float nrm = sqrtf((t1[0] * t1[0] + t1[1] * t1[1]) + t1[2] * t1[2]);
    for (int k = 0; k < 3; ++k) t1[k] = t1[k] / nrm;
    for (int c = 0; c < 4; ++c) {
        memcpy(Rc[c], c < 2 ? R1 : R2, sizeof(R1));
        for (int k = 0; k < 3; ++k) tc[c][k] = (c & 1) ? -t1[k] : t1[k];
    }
}

static float dot3(const float* a, const float* b) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }
static float norm3(const float* a) { return sqrtf(dot3(a, a)); }

static void transform(const float* R, const float* t, const float* x, float* y) {
    for (int r = 0; r < 3; ++r) y[r] = ((R[3 * r] * x[0] + R[3 * r + 1] * x[1]) + R[3 * r + 2] * x[2]) + t[r];
}

/* :728-783 */
static int triangulate1(const float* b1, const float* b2, const float* R, const float* t, float* X) {
    float tr[3], b21[3];
    for (int c = 0; c < 3; ++c) {
        tr[c] = -((R[c] * t[0] + R[3 + c] * t[1]) + R[6 + c] * t[2]);
        b21[c] = (R[c] * b2[0] + R[3 + c] * b2[1]) + R[6 + c] * b2[2];
    }
    const float a00 = dot3(b1, b1), a10 = dot3(b1, b21), a01 = -a10, a11 = -dot3(b21, b21);
    const float r0 = dot3(b1, tr), r1 = dot3(b21, tr);
    const float det = a00 * a11 - a01 * a10;
    if (fabsf(det) < 1e-10f) return 0;
    const float invdet = 1.0f / (a00 * a11 - a10 * a01);
    const float i00 = a11 * invdet, i01 = -a01 * invdet, i10 = -a10 * invdet, i11 = a00 * invdet;
    const float l0 = i00 * r0 + i01 * r1, l1 = i10 * r0 + i11 * r1;
    if (!isfinite(l0) || !isfinite(l1)) return 0;
    for (int c = 0; c < 3; ++c) {
        const float p1 = l0 * b1[c];
        const float p2 = l1 * b21[c] + tr[c];
        X[c] = (p1 + p2) / 2.0f;
    }
    return 1;
}

static float clamp1(float x) { return x < -1.0f ? -1.0f : (1.0f < x ? 1.0f : x); }

/* :837-871 */
static float reproj_error(const float* p, const float* b, int W, int H) {
    const float L = norm3(p);
    if (L < 1e-6f) return 1000.0f;
    const float th_o = atan2f(b[0], b[2]);
    const float ph_o = -asinf(clamp1(b[1]));
    const float u_o = (float)((double)W * ((double)0.5f + (double)th_o / (2.0 * M_PI)));
    const float v_o = (float)((double)H * ((double)0.5f - (double)ph_o / M_PI));
    const float q[3] = {p[0] / L, p[1] / L, p[2] / L};
    const float th_p = atan2f(q[0], q[2]);
    const float ph_p = -asinf(clamp1(q[1]));
    const float u_p = (float)((double)W * ((double)0.5f + (double)th_p / (2.0 * M_PI)));
    const float v_p = (float)((double)H * ((double)0.5f - (double)ph_p / M_PI));
    const float du = u_o - u_p, dv = v_o - v_p;
    return sqrtf(du * du + dv * dv);
}

static int cmp_float(const void* a, const void* b) {
    const float x = *(const float*)a, y = *(const float*)b;
    return x < y ? -1 : (x > y ? 1 : 0);
}

/* returns 0; result->status carries the outcome (VIO_INIT_* codes of include/vio360.h) */
int oracle_mono_init(const float* b1, const float* b2, int n, const int32_t* samples, const oi_params* P,
                     oi_result* res, uint8_t* mask_out, float* points_out) {
    memset(res, 0, sizeof(*res));
    res->best_hypothesis = -1;
    res->pose_candidate = -1;
    res->scale_factor = 1.f;
    uint8_t* mask = (uint8_t*)calloc(n > 0 ? n : 1, 1);
    float* X = (float*)calloc(3 * (size_t)(n > 0 ? n : 1), sizeof(float));
    if (n < 5) {
        res->status = 1;
        goto done;
    }
    /* RANSAC (:483-573) */
    {
        float bestE[9] = {0};
        int best = -1, bc = 0;
        for (int h = 0; h < P->ransac_iterations; ++h) {
            float rows[8][9];
            for (int r = 0; r < 8; ++r) {
                const int i = samples[8 * h + r];
                epi_row(b1 + 3 * i, b2 + 3 * i, rows[r]);
            }
            double G[81], e[9];
            for (int p = 0; p < 9; ++p)
                for (int q = p; q < 9; ++q) {
                    double s = 0.0;
                    for (int r = 0; r < 8; ++r) s += (double)rows[r][p] * (double)rows[r][q];
                    G[p * 9 + q] = G[q * 9 + p] = s;
                }
            null_vector9(G, e);
            float E[9];
            project_essential(e, E);
            int cnt = 0;
            for (int i = 0; i < n; ++i) cnt += epi_err(E, b1 + 3 * i, b2 + 3 * i) < P->ransac_threshold;
            if (cnt > bc) {
                bc = cnt;
                best = h;
                memcpy(bestE, E, sizeof(E));
            }
        }
        res->best_hypothesis = best;
        res->num_inliers = bc;
        for (int i = 0; i < n; ++i) mask[i] = best >= 0 && epi_err(bestE, b1 + 3 * i, b2 + 3 * i) < P->ransac_threshold;
        if (bc < P->min_features) {
            res->status = 2;
            goto done;
        }
    }
    /* refit (:583-616): 64 strided partial sums per entry, then in lane order */
    {
        double G[81], e[9];
        for (int p = 0; p < 9; ++p)
            for (int q = p; q < 9; ++q) {
                double tot = 0.0;
                for (int l = 0; l < 64; ++l) {
                    double s = 0.0;
                    for (int i = l; i < n; i += 64) {
                        if (!mask[i]) continue;
                        float row[9];
                        epi_row(b1 + 3 * i, b2 + 3 * i, row);
                        s += (double)row[p] * (double)row[q];
                    }
                    tot += s;
                }
                G[p * 9 + q] = G[q * 9 + p] = tot;
            }
        null_vector9(G, e);
        project_essential(e, res->E);
    }
    /* RecoverPose (:623-697) */
    float Rc[4][9], tc[4][3];
    pose_candidates(res->E, Rc, tc);
    int bi = -1, bgood = 0;
    for (int c = 0; c < 4; ++c) {
        int good = 0;
        for (int i = 0; i < n; ++i) {
            if (!mask[i]) continue;
            float P3[3], P2[3];
            if (!triangulate1(b1 + 3 * i, b2 + 3 * i, Rc[c], tc[c], P3)) continue;
            const float er = reproj_error(P3, b1 + 3 * i, P->width, P->height);
            transform(Rc[c], tc[c], P3, P2);
            const float ec = reproj_error(P2, b2 + 3 * i, P->width, P->height);
            if (er < 5.0f && ec < 5.0f) ++good;
        }
        res->candidate_good[c] = good;
        if (good > bgood) {
            bgood = good;
            bi = c;
        }
    }
    res->pose_candidate = bi;
    if (bi < 0 || bgood < P->min_features) {
        res->status = 3;
        goto done;
    }
    {
        const float* R = Rc[bi];
        float t[3] = {tc[bi][0], tc[bi][1], tc[bi][2]};
        /* TriangulatePoints (:699-726) */
        int ntri = 0;
        for (int i = 0; i < n; ++i) {
            float* x = X + 3 * i;
            if (triangulate1(b1 + 3 * i, b2 + 3 * i, R, t, x))
                ++ntri;
            else
                x[0] = x[1] = x[2] = 0.f;
        }
        res->num_triangulated = ntri;
        if (ntri < P->min_features) {
            res->status = 4;
            goto done;
        }
        /* ValidateInitialization (:889-995) */
        float sum = 0.f;
        int cnt = 0;
        for (int i = 0; i < n; ++i) {
            if (!mask[i]) continue;
            const float* x = X + 3 * i;
            if ((double)norm3(x) < 1e-6) continue;
            const float er = reproj_error(x, b1 + 3 * i, P->width, P->height);
            if (er > P->max_reprojection_error) continue;
            float x2[3];
            transform(R, t, x, x2);
            const float ec = reproj_error(x2, b2 + 3 * i, P->width, P->height);
            if (ec > P->max_reprojection_error) continue;
            sum += fmaxf(er, ec);
            ++cnt;
        }
        res->num_valid = cnt;
        res->mean_reproj_error = cnt ? sum / (float)cnt : 0.f;
        if (cnt == 0 || cnt < P->min_features) {
            res->status = 5;
            goto done;
        }
        /* NormalizeScale (:997-1048) */
        float* d = (float*)malloc(sizeof(float) * (size_t)n);
        int nd = 0;
        for (int i = 0; i < n; ++i) {
            const float nr = norm3(X + 3 * i);
            if (nr < 1e-6f) continue;
            if (nr > 0.01f) d[nd++] = nr;
        }
        float scale = 1.0f;
        if (nd > 0) {
            qsort(d, nd, sizeof(float), cmp_float);
            const int mid = nd / 2;
            const float med = (nd % 2 == 0) ? (d[mid - 1] + d[mid]) / 2.0f : d[mid];
            scale = 1.0f / med;
        }
        free(d);
        for (int i = 0; i < 3 * n; ++i) X[i] = X[i] * scale;
        for (int k = 0; k < 3; ++k) t[k] = t[k] * scale;
        res->scale_factor = scale;
        memcpy(res->R, R, sizeof(float) * 9);
        memcpy(res->t, t, sizeof(t));
        res->status = 0;
    }
done:
    if (mask_out) memcpy(mask_out, mask, (size_t)n);
    if (points_out) memcpy(points_out, X, sizeof(float) * 3 * (size_t)n);
    free(mask);
    free(X);
    return 0;
}
