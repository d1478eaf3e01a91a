// gwo_xfer.cpp -- copies between device memory and caller memory that may be pageable (the rows gwo_drain,
// gwo_drain_side_output and gwo_snapshot_rows hand out, the columns gwo_submit and gwo_restore take in, the
// stateless helpers' columns).
//
// Pageable host memory is never handed to HIP's copy engine: such a copy runs through a pinned bounce buffer owned
// by the library, in chunks, double-buffered (the DMA of one chunk overlaps the host memcpy of the other). Pinned
// host memory (hipHostMalloc, or a hipHostRegister'ed range -- the Java operator's columns) and device memory are
// copied directly. Round 6: two full GPU-suite runs (r05, r06) reported "illegal memory access" at the drain's
// device-to-host copy into a fresh numpy column with the handle's stream already synchronised and no bounds
// violation in the checked window-step builds; the runtime's pageable path (it pins the caller's
// pages itself above a size threshold) was the one piece of the copy not under the library's control.
#include <hip/hip_runtime.h>

#include <cstring>
#include <mutex>

#include "gwo_handle.h"

namespace gwo {

namespace {

constexpr size_t kHalf = (size_t)4 << 20;   // bytes per bounce half

struct Bounce {
    std::mutex mu;
    int device = -1;
    char *buf = nullptr;   // 2 * kHalf, pinned
    hipEvent_t ev[2] = {nullptr, nullptr};

    hipError_t ready(int dev) {
        if (buf && dev == device) return hipSuccess;
        if (buf) {   // another device than last time: the buffer is pinned for all devices, the events are not
            for (auto &e : ev)
                if (e) (void)hipEventDestroy(e);
            ev[0] = ev[1] = nullptr;
        } else {
            hipError_t e = hipHostMalloc((void **)&buf, 2 * kHalf, hipHostMallocPortable);
            if (e != hipSuccess) {
                buf = nullptr;
                return e;
            }
        }
        for (auto &e : ev) {
            hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
            if (r != hipSuccess) return r;
        }
        device = dev;
        return hipSuccess;
    }
};

Bounce &bounce() {
    static Bounce *b = new Bounce();   // never destroyed: the runtime may be gone at exit
    return *b;
}

}  // namespace

MemKind mem_kind(const void *p) {
    if (!p) return MEM_DEVICE;
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();
        return MEM_PAGEABLE;
    }
    switch (attr.type) {
        case hipMemoryTypeDevice:
        case hipMemoryTypeManaged:
        case hipMemoryTypeUnified:
            return MEM_DEVICE;
        case hipMemoryTypeHost:
            return MEM_PINNED;
        default:
            return MEM_PAGEABLE;
    }
}

// device `src` -> `dst` (any memory), ordered on `s`; complete when this returns
hipError_t copy_out(void *dst, const void *src, size_t bytes, hipStream_t s) {
    if (!bytes) return hipSuccess;
    if (mem_kind(dst) != MEM_PAGEABLE) {
        hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, s);
        return e != hipSuccess ? e : hipStreamSynchronize(s);
    }
    Bounce &B = bounce();
    std::lock_guard<std::mutex> lock(B.mu);
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = B.ready(dev);
    if (e != hipSuccess) return e;
    const size_t nchunks = (bytes + kHalf - 1) / kHalf;
    auto len_of = [&](size_t i) { return std::min(kHalf, bytes - i * kHalf); };
    for (size_t i = 0; i <= nchunks; ++i) {
        if (i < nchunks) {   // chunk i into half i & 1 (that half's previous chunk was copied out at step i - 1)
            char *h = B.buf + (i & 1) * kHalf;
            e = hipMemcpyAsync(h, (const char *)src + i * kHalf, len_of(i), hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipEventRecord(B.ev[i & 1], s);
            if (e != hipSuccess) return e;
        }
        if (i >= 1) {   // chunk i - 1 out of its half while chunk i is in flight
            const size_t j = i - 1;
            e = hipEventSynchronize(B.ev[j & 1]);
            if (e != hipSuccess) return e;
            std::memcpy((char *)dst + j * kHalf, B.buf + (j & 1) * kHalf, len_of(j));
        }
    }
    return hipSuccess;
}

// `src` (any memory) -> device `dst`, ordered on `s`; the caller's memory may be reused when this returns (a
// pinned or device `src` is copied asynchronously and must stay valid until `s` passes the copy, as with
// hipMemcpyAsync)
hipError_t copy_in(void *dst, const void *src, size_t bytes, hipStream_t s) {
    if (!bytes) return hipSuccess;
    if (mem_kind(src) != MEM_PAGEABLE) return hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, s);
    Bounce &B = bounce();
    std::lock_guard<std::mutex> lock(B.mu);
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = B.ready(dev);
    if (e != hipSuccess) return e;
    const size_t nchunks = (bytes + kHalf - 1) / kHalf;
    for (size_t i = 0; i < nchunks; ++i) {
        const size_t len = std::min(kHalf, bytes - i * kHalf);
        char *h = B.buf + (i & 1) * kHalf;
        if (i >= 2) {   // the half's previous chunk must have left it
            e = hipEventSynchronize(B.ev[i & 1]);
            if (e != hipSuccess) return e;
        }
        std::memcpy(h, (const char *)src + i * kHalf, len);
        e = hipMemcpyAsync((char *)dst + i * kHalf, h, len, hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipEventRecord(B.ev[i & 1], s);
        if (e != hipSuccess) return e;
    }
    // both halves free again before the lock is released (the next copy, maybe on another stream, reuses them)
    for (size_t i = nchunks >= 2 ? nchunks - 2 : 0; i < nchunks; ++i) {
        e = hipEventSynchronize(B.ev[i & 1]);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// `src` (device or host memory) -> host `dst` (a library vector): host sources are read by the CPU
hipError_t fetch_host(void *dst, const void *src, size_t bytes, hipStream_t s) {
    if (!bytes) return hipSuccess;
    if (mem_kind(src) != MEM_DEVICE) {
        std::memcpy(dst, src, bytes);
        return hipSuccess;
    }
    return copy_out(dst, src, bytes, s);
}

}  // namespace gwo
