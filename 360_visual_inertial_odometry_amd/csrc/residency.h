// residency.h — co-residency ledger of the library's persistent launches (host side).
//
// Two kinds of launch have workgroups that wait for each other and so must be resident all at once:
// the window-BA cluster route (ph_cluster_kernel: a window's leader and members hand off through
// counters) and the global solver's persistent triangular solves (trsv_*_persistent_kernel).  One such
// launch alone fits the device by construction (ba_cluster_members sizes the cluster grid to the CUs).
// Two of them running at once on different streams of one device — INTEGRATION.md allows one context
// per host thread — could both end up partly placed, each holding CUs that the other's unplaced
// workgroups need; their bounded waits then expire and valid solves come back as VIO_EDEVICE.
//
// A persistent launch therefore reserves its workgroups (one CU each: the cluster kernel takes a whole
// CU; the triangular solves are counted the same way) against the device's capacity before it is
// enqueued.  Reservations of launches still running on OTHER streams count against it (launches on one
// stream run one after another and never compete); a launch that does not fit waits on the host for
// the oldest conflicting launch to finish (its completion event, waited on with the ledger unlocked), then
// is enqueued.  Nothing is added to the stream but one event record per persistent launch.  The ledger is
// per process: two processes sharing a GPU do not see each other's reservations.
#pragma once
#include <hip/hip_runtime.h>

#include <memory>
#include <mutex>

namespace vio360 {

// CUs a persistent launch may occupy on the current device (all but a margin of 8 for other work)
int residency_capacity();

// a launch's completion event, shared by the ledger entry and any guard waiting on it
struct LaunchEvent {
    hipEvent_t ev = nullptr;
    ~LaunchEvent();
};

class ResidencyGuard {
  public:
    // waits until `workgroups` fit beside the persistent launches in flight on other streams of the
    // current device; holds the device's ledger until commit() (or destruction: no reservation).
    // workgroups <= 0 reserves nothing (no lock, no event)
    ResidencyGuard(hipStream_t stream, int workgroups);
    ~ResidencyGuard();
    // after the launch has been enqueued on the stream: its completion ends the reservation (if the
    // event cannot be recorded, commit waits for the stream instead and returns that wait's status)
    hipError_t commit();
    hipError_t status() const { return err_; }
    ResidencyGuard(const ResidencyGuard&) = delete;
    ResidencyGuard& operator=(const ResidencyGuard&) = delete;

  private:
    int dev_ = 0, wgs_ = 0;
    hipStream_t stream_ = nullptr;
    hipError_t err_ = hipSuccess;
    std::unique_lock<std::mutex> lock_;
    std::shared_ptr<LaunchEvent> ev_;
};

}  // namespace vio360
