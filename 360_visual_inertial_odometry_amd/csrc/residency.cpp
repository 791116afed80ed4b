// residency.cpp — the co-residency ledger of persistent launches (residency.h).
#include "residency.h"

#include <vector>

namespace vio360 {

LaunchEvent::~LaunchEvent() {
    if (ev) (void)hipEventDestroy(ev);
}

namespace {

constexpr int kLedgerDevices = 64;

struct Entry {
    hipStream_t stream;
    int wgs;
    std::shared_ptr<LaunchEvent> done;  // recorded after the launch on its stream
};

struct Ledger {
    std::mutex m;
    std::vector<Entry> live;  // launch order
    int cap = 0;
};

Ledger g_ledger[kLedgerDevices];

int device_now() {
    int d = 0;
    return hipGetDevice(&d) == hipSuccess && d >= 0 && d < kLedgerDevices ? d : 0;
}

// drop the entries whose launch has finished (event complete or unusable); an entry's event lives on while
// a waiting guard still holds it
void prune(Ledger& L) {
    size_t k = 0;
    for (size_t i = 0; i < L.live.size(); ++i) {
        const hipError_t q = hipEventQuery(L.live[i].done->ev);
        // (the status is consumed here: it must not stay behind as this thread's last HIP error, where a
        // later hipGetLastError -- ours after a launch, or the caller's -- would report it)
        if (q != hipSuccess) (void)hipGetLastError();
        if (q == hipErrorNotReady) L.live[k++] = std::move(L.live[i]);
    }
    L.live.resize(k);
}

}  // namespace

int residency_capacity() {
    const int dev = device_now();
    Ledger& L = g_ledger[dev];
    std::lock_guard<std::mutex> lk(L.m);
    if (!L.cap) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
        L.cap = cus > 16 ? cus - 8 : cus;
    }
    return L.cap;
}

ResidencyGuard::ResidencyGuard(hipStream_t stream, int workgroups)
    : dev_(device_now()), wgs_(workgroups), stream_(stream) {
    if (wgs_ <= 0) return;  // nothing to reserve: no lock, no event
    const int cap = residency_capacity();
    // the completion event exists before the launch is enqueued, so that commit() only records it
    auto ev = std::make_shared<LaunchEvent>();
    if ((err_ = hipEventCreateWithFlags(&ev->ev, hipEventDisableTiming)) != hipSuccess) {
        ev->ev = nullptr;
        return;
    }
    ev_ = std::move(ev);
    Ledger& L = g_ledger[dev_];
    lock_ = std::unique_lock<std::mutex>(L.m);
    for (;;) {
        prune(L);
        int others = 0;
        std::shared_ptr<LaunchEvent> oldest;
        for (const Entry& e : L.live)
            if (e.stream != stream_) {
                others += e.wgs;
                if (!oldest) oldest = e.done;
            }
        // (a launch larger than the capacity alone is the caller's sizing; it is not held back forever)
        if (!oldest || others + wgs_ <= cap) break;
        // wait for the oldest conflicting launch WITHOUT the ledger: other devices' / fitting launches go on
        lock_.unlock();
        const hipError_t e = hipEventSynchronize(oldest->ev);
        lock_.lock();
        if (e != hipSuccess) {
            // a foreign launch's failure is its own caller's to report: drop its reservation and go on
            (void)hipGetLastError();
            for (size_t i = 0; i < L.live.size(); ++i)
                if (L.live[i].done == oldest) {
                    L.live.erase(L.live.begin() + (long)i);
                    break;
                }
        }
    }
}

hipError_t ResidencyGuard::commit() {
    if (!lock_.owns_lock()) return err_;  // nothing reserved (or the event could not be created)
    Ledger& L = g_ledger[dev_];
    const hipError_t e = hipEventRecord(ev_->ev, stream_);
    if (e == hipSuccess) {
        L.live.push_back(Entry{stream_, wgs_, ev_});
        lock_.unlock();
        return hipSuccess;
    }
    // the launch is enqueued but cannot be tracked: let it finish before anyone else reserves
    (void)hipGetLastError();
    const hipError_t s = hipStreamSynchronize(stream_);
    lock_.unlock();
    return s;
}

ResidencyGuard::~ResidencyGuard() {
    if (lock_.owns_lock()) lock_.unlock();
}

}  // namespace vio360
