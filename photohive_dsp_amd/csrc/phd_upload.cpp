// phd_upload.cpp -- host RGB8 buffers to device memory, pipelined.
//
// The timed region of SURVEY.md 8(d) starts from a u8 HOST buffer.  The
// caller's buffers are pageable (a numpy array, a decoded image).  By default
// they go to the device through the HIP runtime's own pageable path on the
// `h2d` stream (measured 1434 images/s = 51.6 GB/s for 64 x 4000x3000 through
// phd_report_batch_u8, against 1360 for the ring below).  PHD_UPLOAD=staged
// selects an explicit ring: each image is cut into 16 MB chunks that rotate
// through pinned slots, copy threads filling slot j while the DMA engine sends
// slot j - 1.
//
// phd_report_batch_u8 runs the uploads of the next same-size group on an
// uploader thread while the current group's reports compute (two device
// staging buffers), so the H2D traffic overlaps the GPU work.
// PHD_UPLOAD_STREAMS=2 sends a group's odd images on a second stream from a
// second thread (two pageable copies in flight): 1442-1453 against 1386-1439
// images/s alone (tools/host_overlap.py), but 860-909 against 1375-1414 in
// bench.py's host_buffer leg, so one stream is the default.
#include <algorithm>
#include <cstring>
#include <thread>

#include <unistd.h>

#include "phd_host.h"

namespace phd {

namespace {
constexpr size_t kSlotBytes = (size_t)16 << 20;
constexpr int kSlots = 8;
}  // namespace

namespace {
std::mutex g_copy_mu;
HostPool* g_copy = nullptr;
pid_t g_copy_owner = 0;
}  // namespace

HostPool* copy_pool() {
    // the palette decisions own host_pool(); the copies get their own threads
    std::lock_guard<std::mutex> lk(g_copy_mu);
    if (!g_copy || g_copy_owner != getpid()) {
        const unsigned hc = std::thread::hardware_concurrency();
        g_copy = new HostPool(hc > 2 ? (int)std::min(hc - 1, 7u) : 0);
        g_copy_owner = getpid();
    }
    return g_copy;
}

void stop_copy_pool() {
    std::lock_guard<std::mutex> lk(g_copy_mu);
    if (g_copy && g_copy_owner == getpid()) {
        g_copy->stop();
        delete g_copy;
    }
    g_copy = nullptr;
}

int copy_pool_threads() {
    std::lock_guard<std::mutex> lk(g_copy_mu);
    return g_copy && g_copy_owner == getpid() ? g_copy->size() : 0;
}

static bool staged_upload() {
    static const bool staged = phd_knob("PHD_UPLOAD") && !strcmp(phd_knob("PHD_UPLOAD"), "staged");
    return staged;
}

// The streams and events every upload path uses.  c->h2d is set last, so a
// failed setup leaves the context without it and the next call retries; each
// failure names itself.
bool upload_init(Context* c) {
    if (c->h2d) return true;
    hipStream_t h2d = nullptr;
    if (!c->h2d2 && hipStreamCreateWithFlags(&c->h2d2, hipStreamNonBlocking) != hipSuccess) {
        c->h2d2 = nullptr;
        set_error("upload setup: second upload stream creation failed");
        return false;
    }
    if (!c->ev_h2d2 && hipEventCreateWithFlags(&c->ev_h2d2, device_event_flags()) != hipSuccess) {
        c->ev_h2d2 = nullptr;
        set_error("upload setup: upload event creation failed");
        return false;
    }
    for (auto& e : c->ev_up)
        if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
            e = nullptr;
            set_error("upload setup: upload event creation failed");
            return false;
        }
    if (hipStreamCreateWithFlags(&h2d, hipStreamNonBlocking) != hipSuccess) {
        set_error("upload setup: upload stream creation failed");
        return false;
    }
    c->h2d = h2d;
    return true;
}

// The pinned slot ring of the staged path (PHD_UPLOAD=staged only: the default
// pageable path never touches it, so it is not allocated there).
static bool staged_init(Context* c, std::string* why) {
    if (c->h2d_slots) return true;
    if (c->ev_slot.size() != (size_t)kSlots) c->ev_slot.assign(kSlots, nullptr);
    for (auto& e : c->ev_slot)
        if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
            e = nullptr;
            *why = "upload setup: slot event creation failed";
            return false;
        }
    uint8_t* slots = nullptr;
    if (hipHostMalloc((void**)&slots, kSlotBytes * kSlots, hipHostMallocDefault) != hipSuccess) {
        *why = "upload setup: pinned slot ring allocation failed";
        return false;
    }
    c->slot_used.assign(kSlots, 0);
    c->next_slot = 0;
    c->h2d_slots = slots;
    return true;
}

// Enqueue the transfer of `bytes` contiguous host bytes to d_dst on c->h2d.
// Returns once every chunk has been copied into a pinned slot (the caller's
// buffer is no longer read); the DMA may still be running.

int upload_streams() {
    static const int n = phd_knob("PHD_UPLOAD_STREAMS") ? std::min(2, std::max(1, atoi(phd_knob("PHD_UPLOAD_STREAMS"))))
                                                      : 1;
    return staged_upload() ? 1 : n;
}

bool upload_async(Context* c, uint8_t* d_dst, const uint8_t* src, size_t bytes, std::string* why, hipStream_t s) {
    if (!staged_upload()) {   // the HIP runtime's own pageable path (faster, measured)
        const hipStream_t us = s ? s : c->h2d;
        const hipError_t e = hipMemcpyAsync(d_dst, src, bytes, hipMemcpyHostToDevice, us);
        if (e != hipSuccess) *why = std::string("upload failed: ") + hipGetErrorString(e);
        return e == hipSuccess && hipStreamSynchronize(us) == hipSuccess;
    }
    if (!staged_init(c, why)) return false;
    HostPool* pool = copy_pool();
    for (size_t off = 0; off < bytes; off += kSlotBytes) {
        const int s = c->next_slot;
        c->next_slot = (c->next_slot + 1) % kSlots;
        if (c->slot_used[s] && hipEventSynchronize(c->ev_slot[s]) != hipSuccess) {
            *why = "upload: slot event failed";
            return false;
        }
        const size_t n = std::min(kSlotBytes, bytes - off);
        uint8_t* slot = c->h2d_slots + (size_t)s * kSlotBytes;
        constexpr size_t piece = (size_t)1 << 20;
        const int np = (int)((n + piece - 1) / piece);
        pool->parallel_for(np, [&](int k) {
            const size_t o = (size_t)k * piece;
            memcpy(slot + o, src + off + o, std::min(piece, n - o));
        });
        hipError_t e = hipMemcpyAsync(d_dst + off, slot, n, hipMemcpyHostToDevice, c->h2d);
        if (e == hipSuccess) e = hipEventRecord(c->ev_slot[s], c->h2d);
        if (e != hipSuccess) {
            *why = std::string("upload failed: ") + hipGetErrorString(e);
            return false;
        }
        c->slot_used[s] = 1;
    }
    return true;
}

}  // namespace phd
