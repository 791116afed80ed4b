// ba_global.h — device argument block and launchers of the global-BA path (ba_global.hip), driven
// by the host LM loop in ba_global_host.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "vio360.h"

namespace vio360 {

struct GbaArgs {
    int K, L, N;
    int P;            // free poses (pose blocks of the reduced system)
    int nf, nfp;      // reduced size 6P and its 64-padded size
    double cols, rows, huber, chi2_thr;
    double Lw[4], info[4];
    // inputs (landmark-sorted observations)
    const double* pose_raw;   // [K][24] raw R_init t_init R_cb t_cb
    const int* pose_f;        // [K] f-offset (6 * block) or -1
    const int* pose_of_block; // [P] keyframe of pose block p
    const uint8_t* lm_var;    // [L]
    const uint8_t* lm_marg;   // [L]
    const int* lm_ptr;        // [L+1]
    const int* obs_kf;        // [N]
    const int* obs_lm;        // [N]
    const float* obs_uv;      // [N][2]
    const int* kf_ptr;        // [K+1]
    const int* kf_obs;        // [N]
    // Schur contributions sorted by destination block (pa >= pb)
    long long n_dest;
    const int* dest_a;        // [n_dest]
    const int* dest_b;
    const int* dest_ptr;      // [n_dest+1]
    const int* contrib_a;     // [n_contrib] observation indices
    const int* contrib_b;
    // state
    double* pinit;            // [K][24]
    double* pc;               // [K][36]
    double* x_pose;           // [K][6]
    double* x_lm;             // [L][3]
    double* c_pose;
    double* c_lm;
    double* r;                // [2][N]
    double* jp;               // [12][N]
    double* jl;               // [6][N]
    double* V;                // [6][L]
    double* gl;               // [3][L]
    double* sl;               // [3][L]
    double* Vi;               // [6][L]
    double* yl;               // [3][L]
    double* U;                // [K][27]
    double* gf;               // [nfp]
    double* colsq_f;
    double* sf;
    double* Df;
    double* bf;               // rhs (consumed by the forward substitution)
    double* yv;               // forward result
    double* xf;               // reduced-system solution
    double* Wo;               // [N][18]
    double* Yo;               // [N][18]
    double* S;                // [nfp][nfp]
    double* Linv;             // [nfp/64 + 2][64][64]: the inverse diagonal blocks + the chained Cholesky's scratch
    hipStream_t side;         // look-ahead stream of the Cholesky (nullptr: plain schedule)
    hipEvent_t ev[2];
    int* flags;               // [32 (3 nfp/64 + 1)] triangular-solve flags, one per 128 B (+ timeout word), Cholesky step flags
    // RunVIBA beyond one window (Optimizer.cpp:493-724): the velocities and the shared biases follow the
    // pose blocks in the reduced system (f = np + imu index, the oracle's order); the IMU factors'
    // pose Jacobians are zero in the reference (Factors.cpp:1326-1485), so the reduced system is
    // blockdiag(pose Schur complement, IMU normal equations) and the landmarks never couple to it
    int is_vi;
    int np, ni;               // 6P pose rows, nf - np IMU rows
    double gravity[3];
    const vio_preint* preint;       // [K]
    const uint8_t* preint_valid;    // [K]
    const int* vel_f;         // [K] f-offset of velocity k or -1
    int bg_f, ba_f;           // f-offsets of the biases (-1: no IMU factor)
    double* sqi;              // [K][81] sqrt-information of each factor
    double* x_vel;            // [K][3]
    double* c_vel;
    double* x_bias;           // [6] bg, ba
    double* c_bias;
    double* imuJ;             // [K][108] Jacobian 9x12 [vi | bg | ba | vj] at the linearisation point
    double* imur;             // [K][9] residual there
    double* imu_cost;         // [K] per-factor cost (scratch of the fixed-order sum)
    double* Himu;             // [ni][ni] J^T J of the IMU factors (imu-space)
};
// GbaArgs crosses translation units (ba_global_host.cpp fills it; ba_global.hip and ba_kernel.hip's
// gba_imu.inc read it): its layout is pinned here, in every TU that includes this header, and each of
// those TUs exports its compiled-in signature (gba_layout_sig_*) for the runtime cross-check in
// vio_ctx_create.  Change a member => update these numbers (and the build rebuilds every user).
static_assert(sizeof(GbaArgs) == 640, "GbaArgs layout changed: update the pinned size");
static_assert(offsetof(GbaArgs, flags) == 488 && offsetof(GbaArgs, is_vi) == 496 &&
              offsetof(GbaArgs, S) == 448 && offsetof(GbaArgs, Himu) == 632, "GbaArgs offsets changed");
constexpr uint64_t gba_layout_sig() {
    return (uint64_t)sizeof(GbaArgs) << 48 | (uint64_t)offsetof(GbaArgs, flags) << 32 |
           (uint64_t)offsetof(GbaArgs, is_vi) << 16 | (uint64_t)offsetof(GbaArgs, Himu);
}

// the word a timed-out inter-workgroup wait of the Cholesky / triangular solves sets (cleared by
// gba_reset_timeout before every factorisation, outside the captured graph); nonzero after a step means a
// device fault, not a failed factorisation
inline int* gba_timeout_word(const GbaArgs& A) { return A.flags ? A.flags + 32 * 2 * (size_t)(A.nfp / 64) : nullptr; }

hipError_t gba_launch_setup(const GbaArgs& A, hipStream_t s);
// mode 0 cost of active blocks, 1 + Jacobians, 2 cost of the constant blocks; out[0] = cost
hipError_t gba_launch_eval(const GbaArgs& A, const double* xp, const double* xl, int mode, double* partial,
                           double* out, hipStream_t s);
hipError_t gba_launch_linearise(const GbaArgs& A, int first, double* partial, double* out_gmax, hipStream_t s);
hipError_t gba_launch_step_prep(const GbaArgs& A, double radius, double* partial, double* out_bad, hipStream_t s);
hipError_t gba_cholesky_attributes();
hipError_t gba_reset_timeout(const GbaArgs& A, hipStream_t s);
hipError_t gba_launch_cholesky(const GbaArgs& A, int* fail, hipStream_t s);
hipError_t gba_launch_solve(const GbaArgs& A, hipStream_t s);
// workgroups of the persistent triangular solves gba_launch_solve enqueues (0: the per-step kernels), for
// the co-residency ledger (residency.h)
int gba_solve_persistent_wgs(const GbaArgs& A);
hipError_t gba_launch_backsub(const GbaArgs& A, double* partial, double* out_nonfinite, hipStream_t s);
hipError_t gba_launch_model(const GbaArgs& A, double* partial, double* out3, hipStream_t s);
// VIBA terms (ba_kernel.hip, next to the window solver's IMU factor code)
hipError_t gba_imu_launch_setup(const GbaArgs& A, hipStream_t s);
// IMU cost at (A.pc, xv, xb) into out[0]; with want_jac the Jacobians / residuals into imuJ / imur
hipError_t gba_imu_launch_eval(const GbaArgs& A, const double* xv, const double* xb, int want_jac, double* out,
                               hipStream_t s);
// IMU normal equations, f-space gradient / column norms (/ Jacobi scale when first) and out[0] = the
// gradient max-norm over the IMU parameters
hipError_t gba_imu_launch_linearise(const GbaArgs& A, int first, double* out_gmax, hipStream_t s);
// rows [np, nf) of the reduced system: sHs + D^2 on the IMU block, zero against the poses
hipError_t gba_imu_launch_system(const GbaArgs& A, hipStream_t s);
// IMU model change, velocity / bias candidates and their step / parameter norms into out3[0..2]
hipError_t gba_imu_launch_model(const GbaArgs& A, double* out3, hipStream_t s);
hipError_t gba_launch_post(const GbaArgs& A, double* chi2, uint8_t* outl, uint8_t* bad, double* partial, double* out3,
                           hipStream_t s);

}  // namespace vio360
