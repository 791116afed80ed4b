// residency.cpp — the co-residency ledger of persistent launches (residency.h).
#include "residency.h"

#include <vector>

namespace vio360 {
namespace {

constexpr int kLedgerDevices = 64;

struct Entry {
    hipStream_t stream;
    int wgs;
    hipEvent_t done;  // recorded after the launch on its stream
};

struct Ledger {
    std::mutex m;
    std::vector<Entry> live;        // launch order
    std::vector<hipEvent_t> spare;  // completed entries' events, reused
    int cap = 0;
};

Ledger g_ledger[kLedgerDevices];

int device_now() {
    int d = 0;
    return hipGetDevice(&d) == hipSuccess && d >= 0 && d < kLedgerDevices ? d : 0;
}

// drop the entries whose launch has finished (event complete or unusable)
void prune(Ledger& L) {
    size_t k = 0;
    for (size_t i = 0; i < L.live.size(); ++i) {
        const hipError_t q = hipEventQuery(L.live[i].done);
        // (the status is consumed here: it must not stay behind as this thread's last HIP error, where a
        // later hipGetLastError -- ours after a launch, or the caller's -- would report it)
        if (q != hipSuccess) (void)hipGetLastError();
        if (q == hipErrorNotReady) L.live[k++] = L.live[i];
        else L.spare.push_back(L.live[i].done);
    }
    L.live.resize(k);
}

}  // namespace

int residency_capacity() {
    Ledger& L = g_ledger[device_now()];
    std::lock_guard<std::mutex> lk(L.m);
    if (!L.cap) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device_now()) != hipSuccess) return 0;
        L.cap = cus > 16 ? cus - 8 : cus;
    }
    return L.cap;
}

ResidencyGuard::ResidencyGuard(hipStream_t stream, int workgroups)
    : dev_(device_now()), wgs_(workgroups), stream_(stream) {
    const int cap = residency_capacity();
    Ledger& L = g_ledger[dev_];
    lock_ = std::unique_lock<std::mutex>(L.m);
    for (;;) {
        prune(L);
        int others = 0;
        const Entry* oldest = nullptr;
        for (const Entry& e : L.live)
            if (e.stream != stream_) {
                others += e.wgs;
                if (!oldest) oldest = &e;
            }
        // (a launch larger than the capacity alone is the caller's sizing; it is not held back forever)
        if (!oldest || others + wgs_ <= cap) break;
        const hipError_t e = hipEventSynchronize(oldest->done);
        if (e != hipSuccess) {
            err_ = e;
            break;
        }
    }
}

hipError_t ResidencyGuard::commit() {
    if (!lock_.owns_lock()) return err_;
    Ledger& L = g_ledger[dev_];
    hipEvent_t ev = nullptr;
    if (!L.spare.empty()) {
        ev = L.spare.back();
        L.spare.pop_back();
    } else if ((err_ = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) {
        lock_.unlock();
        return err_;
    }
    err_ = hipEventRecord(ev, stream_);
    if (err_ == hipSuccess) L.live.push_back(Entry{stream_, wgs_, ev});
    else L.spare.push_back(ev);
    lock_.unlock();
    return err_;
}

ResidencyGuard::~ResidencyGuard() {
    if (lock_.owns_lock()) lock_.unlock();
}

}  // namespace vio360
