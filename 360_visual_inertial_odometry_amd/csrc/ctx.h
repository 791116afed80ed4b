// ctx.h — vio_ctx: device + stream + grow-only device scratch (host side of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <memory>
#include <string>
#include <vector>

#include "vio360.h"

struct vio_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string last_error;
    // grow-only device buffers keyed by slot
    std::vector<void*> bufs;
    std::vector<size_t> caps;
    // grow-only pinned host staging buffers keyed by slot
    std::vector<void*> hbufs;
    std::vector<size_t> hcaps;
    // IMU preintegration kernel timing (created on first use)
    hipEvent_t imu_ev[2] = {nullptr, nullptr};
    float imu_ms = -1.f;
    // triangulation kernel timing (created on first use)
    hipEvent_t tri_ev[2] = {nullptr, nullptr};
    // INTER_AREA resize kernel timing (created on first use)
    hipEvent_t rsz_ev[2] = {nullptr, nullptr};
    // monocular initialisation kernels timing (created on first use)
    hipEvent_t init_ev[2] = {nullptr, nullptr};
    // window-BA execution route (vio_ctx_set_ba_route)
    int ba_route = VIO_BA_ROUTE_AUTO;
    // global-BA state kept between solves (ba_global_host.cpp GbaCache: look-ahead stream, captured graph)
    std::shared_ptr<void> gba_cache;
};

namespace vio360 {

void set_error(vio_ctx* ctx, const std::string& msg);
int hip_fail(vio_ctx* ctx, hipError_t e, const char* what);
// device buffer of at least `bytes` for slot `slot` (contents undefined); nullptr on failure
void* ctx_buffer(vio_ctx* ctx, int slot, size_t bytes);
// pinned host buffer of at least `bytes` for slot `slot` (contents undefined); nullptr on failure
void* ctx_host_buffer(vio_ctx* ctx, int slot, size_t bytes);
// scratch slots owned by vio_imu_preintegrate
enum { kSlotImuData = 8, kSlotImuIntervals = 9, kSlotImuOut = 10 };
// scratch slots owned by vio_triangulate
enum { kSlotTriIn = 11, kSlotTriOut = 12 };
// scratch slots owned by erp_resize_area
enum { kSlotResizeSrc = 13, kSlotResizeDst = 14 };
// staging of vio_ba_batch_pack to host memory
enum { kSlotRecords = 15 };
// vio_imu_init_solve inputs, outputs and per-problem scratch
enum { kSlotImuInit = 16 };
// vio_mono_init_solve inputs, outputs and scratch
enum { kSlotMonoInit = 17 };
// vio_lie_eval inputs and outputs
enum { kSlotLie = 18 };
// the one-shot window solves' arena (vio_ba_solve[_batched]: inputs, outputs, workspace)
enum { kSlotBaSolve = 19 };
// the global BA solves' arena (inputs, outputs, the dense reduced system and the rest of the state)
enum { kSlotGbaSolve = 20 };
// pinned host slots: the one-shot solves' input image and every BA download's outputs image
enum { kHostSlotBaIn = 0, kHostSlotBaOut = 1, kHostSlotGba = 2 };

// Selects a device for the rest of the enclosing scope and restores the calling thread's current
// device on exit, so a C-ABI call never leaves the caller's thread on the context's device (a process
// that also drives other GPUs, e.g. through torch, keeps its own current device).
struct DeviceScope {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceScope(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) err = hipSetDevice(dev);
        else prev = -1;  // nothing to restore
    }
    ~DeviceScope() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceScope(const DeviceScope&) = delete;
    DeviceScope& operator=(const DeviceScope&) = delete;
};
#define VIO_DEVICE(ctx)                     \
    DeviceScope _vio_dev_scope((ctx)->device); \
    VIO_HIP(ctx, _vio_dev_scope.err)

#define VIO_HIP(ctx, expr)                                  \
    do {                                                    \
        hipError_t _e = (expr);                             \
        if (_e != hipSuccess) return hip_fail(ctx, _e, #expr); \
    } while (0)

}  // namespace vio360
