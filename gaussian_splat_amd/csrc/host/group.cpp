// group.cpp — multi-GPU frames from one host process (gs_create_sharded,
// SURVEY §8(b)/(e)).  No reference counterpart: the reference renders on one
// Metal device.
//
// A group owns one shard handle per GPU: contiguous splat-index ranges of the
// (cropped) scene, made with gs_create_subset.  A frame runs the same per-rank
// C-ABI steps as the one-process-per-GPU path (gaussian_splat_amd/
// distributed.py), driven here by one worker thread per rank:
//
//   rows  (default; the frame is bit-identical to one GPU's)
//     gs_shard_project -> all-to-all of exchange records -> gs_shard_render
//     -> each rank's band of bin rows into the frame on devices[0]
//     With two frames in flight (gs_group_set_frames_in_flight 2,
//     gs_group_render_pipelined) a call projects frame k and starts its
//     all-to-all on the ranks' exchange streams (a communicator set of its
//     own), then renders frame k-1, whose records arrived under frame k's
//     projection, and gathers it on the ranks' gather streams: the link
//     time of one frame hides under the other's compute.
//   slabs (the north star's depth slabs + RGBA reduce)
//     gs_slab_project -> all-reduce of the depth histogram -> gs_slab_pack
//     -> all-to-all -> gs_slab_render -> all-gather of the transmittance
//     -> gs_slab_composite -> reduce (SUM) of the contributions on devices[0]
//
// Transport: RCCL over xGMI (ncclCommInitAll, grouped ncclSend/ncclRecv,
// ncclAllReduce / ncclAllGather / ncclReduce) when every rank has its own
// device, loaded at gs_group_initialize; GS_TRANSPORT_COPY moves the same
// bytes with peer copies (hipMemcpyPeerAsync) and sums slab contributions
// on devices[0] in rank order — the only choice when ranks share a device
// (virtual ranks on one GPU, the tests' configuration).
//
// Failure handling (the reference's only recovery is
// instanced_splat_renderer.mm:319-336): every host wait of a group is
// bounded (gs_group_set_timeout, default GS_COMM_TIMEOUT_MS or 60 s) and,
// under RCCL, polls ncclCommGetAsyncError; a peer error or an expired wait
// aborts every communicator (ncclCommAbort) and fails the frame with
// GS_ERR_COMM.  The group is then unusable (later calls return GS_ERR_COMM).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../kernels/gs_kernels.h"
#include "comm_set.h"
#include "gs_internal.h"
#include "gsplat.h"

namespace {

gs_status gfail(gs_status s, const std::string& msg) {
    gs_set_last_error(msg);
    return s;
}

#define GG_HIP(expr)                                                                               \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess)                                                                      \
            return gfail(e_ == hipErrorOutOfMemory ? GS_ERR_OOM : GS_ERR_DEVICE,                   \
                         std::string(#expr) + ": " + hipGetErrorString(e_));                       \
    } while (0)

// RCCL entry points, resolved at gs_group_initialize (no link-time
// dependency: a process that never builds an RCCL group never loads it).
struct Rccl {
    void* so = nullptr;
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclReduce) reduce = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    decltype(&ncclCommGetAsyncError) async_error = nullptr;
    decltype(&ncclCommAbort) comm_abort = nullptr;
    bool shared_devices = false;  // ranks may share a device (the test stub, tests/cpp/rccl_stub.hip)
    bool load(std::string* why) {
        if (so) return true;
        // GS_RCCL_LIB (tests only): the one library to load instead of RCCL,
        // e.g. the stub that runs this transport's code on a one-GPU box
        const char* over = std::getenv("GS_RCCL_LIB");
        if (over && *over) {
            so = dlopen(over, RTLD_NOW | RTLD_LOCAL);
        } else {
            for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
                so = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
                if (so) break;
            }
        }
        if (!so) {
            *why = std::string("RCCL not loadable: ") + dlerror();
            return false;
        }
        bool ok = true;
        auto sym = [&](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(so, name));
            ok = ok && fn != nullptr;
        };
        sym(comm_init_all, "ncclCommInitAll");
        sym(comm_destroy, "ncclCommDestroy");
        sym(group_start, "ncclGroupStart");
        sym(group_end, "ncclGroupEnd");
        sym(send, "ncclSend");
        sym(recv, "ncclRecv");
        sym(all_reduce, "ncclAllReduce");
        sym(all_gather, "ncclAllGather");
        sym(reduce, "ncclReduce");
        sym(error_string, "ncclGetErrorString");
        sym(async_error, "ncclCommGetAsyncError");
        sym(comm_abort, "ncclCommAbort");
        if (!ok) *why = "RCCL: missing symbols";
        using SharedFn = int (*)();
        const auto sh = reinterpret_cast<SharedFn>(dlsym(so, "gs_rccl_stub_shared_devices"));
        shared_devices = sh && sh() == 1;
        return ok;
    }
};
Rccl g_rccl;

#define GG_NCCL(expr)                                                                                \
    do {                                                                                             \
        ncclResult_t r_ = (expr);                                                                    \
        if (r_ != ncclSuccess)                                                                       \
            return gfail(GS_ERR_COMM, std::string(#expr) + ": " + g_rccl.error_string(r_));          \
    } while (0)

// One worker thread per rank; run(f) executes f(rank) on every worker and
// returns once all are done.
class Pool {
public:
    explicit Pool(int n) {
        for (int i = 0; i < n; ++i) th_.emplace_back([this, i] { loop(i); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> l(mu_);
            quit_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void run(const std::function<void(int)>& f) {
        std::unique_lock<std::mutex> l(mu_);
        job_ = &f;
        pending_ = (int)th_.size();
        ++gen_;
        cv_.notify_all();
        done_.wait(l, [this] { return pending_ == 0; });
        job_ = nullptr;
    }

private:
    void loop(int i) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)>* job;
            {
                std::unique_lock<std::mutex> l(mu_);
                cv_.wait(l, [&] { return quit_ || gen_ != seen; });
                if (quit_) return;
                seen = gen_;
                job = job_;
            }
            (*job)(i);
            std::lock_guard<std::mutex> l(mu_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* job_ = nullptr;
    uint64_t gen_ = 0;
    int pending_ = 0;
    bool quit_ = false;
};

struct DevMem {
    void* ptr = nullptr;
    size_t bytes = 0;
    int dev = -1;
    void release() {
        if (ptr) {
            (void)hipSetDevice(dev);
            (void)hipFree(ptr);
        }
        ptr = nullptr;
        bytes = 0;
    }
    hipError_t reserve(int device, size_t want) {
        if (want <= bytes && device == dev) return hipSuccess;
        release();
        dev = device;
        size_t b = std::max<size_t>(want + want / 8, 256);
        hipError_t e = hipSetDevice(device);
        if (e == hipSuccess) e = hipMalloc(&ptr, b);
        if (e == hipSuccess) bytes = b;
        return e;
    }
    template <typename T>
    T* as() const { return static_cast<T*>(ptr); }
};

struct Rank {
    gs_handle* h = nullptr;
    int dev = 0;
    int64_t base = 0;
    hipStream_t st = nullptr;  // rank 0: the caller's stream during a frame
    bool own_stream = false;
    hipEvent_t ev_ready = nullptr, ev_done = nullptr;
    DevMem send, recv, band, hist, tloc, tall, contrib, stage;
    std::vector<int64_t> counts;  // records to each rank
    // two frames in flight (rows): compute, exchange and gather streams of the
    // rank, the exchange buffers per frame slot, and the events between them:
    // ev_proj (a frame's records are packed), ev_xdone[s] (slot s's all-to-all
    // is done: its send buffer is free, its receive buffer full), ev_rdone[s]
    // (slot s's records are rendered: its receive buffer is free), ev_gdone
    // (the band's gather is done: the band is free)
    hipStream_t cs = nullptr, xs = nullptr, gs = nullptr;
    DevMem psend[2], precv[2];
    std::vector<int64_t> pcounts[2];
    hipEvent_t ev_proj = nullptr, ev_xdone[2] = {}, ev_rdone[2] = {}, ev_gdone = nullptr;
    gs_status status = GS_OK;
    std::string error;
};

}  // namespace

struct gs_group {
    gs_options opt{};
    int world = 1;
    int64_t n = 0;
    int scheme = GS_SCHEME_ROWS;
    bool replicated = false;  // every rank holds the whole scene (bands only)
    int transport = GS_TRANSPORT_COPY;
    bool initialized = false;
    std::vector<Rank> r;
    std::vector<ncclComm_t> comms;
    Pool* pool = nullptr;
    hipEvent_t frame_done = nullptr;  // on devices[0]: everything of the last frame
    DevMem fb;                        // host-output frames
    int64_t timeout_ms = 60000;       // bound of every host wait (gs_group_set_timeout)
    bool timeout_set = false;         // set by gs_group_set_timeout (GS_COMM_TIMEOUT_MS then ignored)
    bool failed = false;              // communicators aborted: the group is unusable
    // two frames in flight (rows scheme, gs_group_render_pipelined)
    int frames_in_flight = 1;
    bool pipe_ready = false;          // the ranks' pipeline streams and events exist
    std::vector<ncclComm_t> xcomms;   // the all-to-all's own communicators (RCCL)
    int pslot = 0;                    // exchange slot of the next projected frame
    struct Pending {                  // the frame whose records are in flight
        bool on = false;
        int slot = 0, width = 0, height = 0;
        std::vector<int64_t> nrec;
    } pend;
    ~gs_group() {
        delete pool;
        for (auto& k : r) {
            if (k.dev >= 0) (void)hipSetDevice(k.dev);
            for (hipStream_t q : {k.cs, k.xs, k.gs})
                if (q) (void)hipStreamSynchronize(q);
            for (DevMem* m : {&k.send, &k.recv, &k.band, &k.hist, &k.tloc, &k.tall, &k.contrib, &k.stage, &k.psend[0],
                              &k.psend[1], &k.precv[0], &k.precv[1]})
                m->release();
            if (k.own_stream && k.st) (void)hipStreamDestroy(k.st);
            if (k.ev_ready) (void)hipEventDestroy(k.ev_ready);
            if (k.ev_done) (void)hipEventDestroy(k.ev_done);
            for (hipStream_t q : {k.cs, k.xs, k.gs})
                if (q) (void)hipStreamDestroy(q);
            for (hipEvent_t e : {k.ev_proj, k.ev_xdone[0], k.ev_xdone[1], k.ev_rdone[0], k.ev_rdone[1], k.ev_gdone})
                if (e) (void)hipEventDestroy(e);
            gs_destroy(k.h);
        }
        // (a failure has aborted and cleared every handle already)
        gscomm::destroy_all(comms, [](ncclComm_t c) { return g_rccl.comm_destroy(c); });
        gscomm::destroy_all(xcomms, [](ncclComm_t c) { return g_rccl.comm_destroy(c); });
        if (frame_done) (void)hipEventDestroy(frame_done);
        fb.release();
    }
};

namespace {

// f(rank) on every rank's worker (device set); the first failure's status and
// gs_last_error text are passed to the caller's thread.
gs_status run_ranks(gs_group* g, const std::function<gs_status(Rank&, int)>& f) {
    std::function<void(int)> job = [&](int i) {
        Rank& k = g->r[(size_t)i];
        if (hipSetDevice(k.dev) != hipSuccess) {
            k.status = GS_ERR_DEVICE;
            k.error = "hipSetDevice";
            return;
        }
        // nothing may escape a worker thread (std::terminate): allocation
        // failures map to GS_ERR_OOM, anything else to GS_ERR_DEVICE
        try {
            k.status = f(k, i);
            k.error = k.status == GS_OK ? std::string() : std::string(gs_last_error());
        } catch (const std::bad_alloc&) {
            k.status = GS_ERR_OOM;
            k.error = "out of host memory";
        } catch (const std::exception& e) {
            k.status = GS_ERR_DEVICE;
            k.error = e.what();
        } catch (...) {
            k.status = GS_ERR_DEVICE;
            k.error = "unknown exception";
        }
    };
    g->pool->run(job);
    for (auto& k : g->r)
        if (k.status != GS_OK) return gfail(k.status, "rank: " + k.error);
    return GS_OK;
}

// Abort every communicator after a peer error or an expired wait.
gs_status comm_failure(gs_group* g, const std::string& why) {
    if (g->transport == GS_TRANSPORT_RCCL) {
        gscomm::abort_all(g->comms, [](ncclComm_t c) { return g_rccl.comm_abort(c); });
        gscomm::abort_all(g->xcomms, [](ncclComm_t c) { return g_rccl.comm_abort(c); });
    }
    g->failed = true;
    return gfail(GS_ERR_COMM, why);
}

// Host wait for `ev` (recorded on a stream of device `dev`), bounded by the
// group's timeout; under RCCL each poll also checks every communicator's
// asynchronous error state.
gs_status wait_bounded(gs_group* g, int dev, hipEvent_t ev, const char* what) {
    GG_HIP(hipSetDevice(dev));
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned spin = 0;; ++spin) {
        const hipError_t e = hipEventQuery(ev);
        if (e == hipSuccess) return GS_OK;
        if (e != hipErrorNotReady) GG_HIP(e);
        if (g->transport == GS_TRANSPORT_RCCL)
            for (const auto* set : {&g->comms, &g->xcomms})
                for (ncclComm_t c : *set) {
                    ncclResult_t ae = ncclSuccess;
                    if (c && g_rccl.async_error(c, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress)
                        return comm_failure(g, std::string(what) + ": RCCL peer error: " + g_rccl.error_string(ae));
                }
        const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
        if (ms > g->timeout_ms)
            return comm_failure(g, std::string(what) + ": no completion within " + std::to_string(g->timeout_ms) + " ms");
        if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

// Row ownership of the default table (gs_shard_set_rows not used by groups):
// rank d owns bin rows [d*R/world, (d+1)*R/world).
void owned_rows(int H, int world, int d, int* row0, int* nrows) {
    const int R = (H + gs::kBin - 1) / gs::kBin;
    *row0 = (int)((int64_t)d * R / world);
    *nrows = (int)((int64_t)(d + 1) * R / world) - *row0;
}

// All-to-all of the exchange records: rank d receives, in source-rank order,
// the records every rank packed for it.  Returns the received counts.
// One transfer of the all-to-all: n records from src's send buffer at
// record offset soff into dst's receive buffer at roff.  Both transports run
// this same plan, so the peer-copy path the one-GPU tests exercise checks
// the offsets the RCCL path sends and receives at.
struct Xfer {
    int src, dst;
    int64_t soff, roff, n;
};

// counts[s][d]: records rank s packed for rank d (grouped by destination in
// s's send buffer); d receives them in source-rank order.
std::vector<Xfer> exchange_plan(const std::vector<std::vector<int64_t>>& counts) {
    const int W = (int)counts.size();
    std::vector<Xfer> plan;
    for (int s = 0; s < W; ++s)
        for (int d = 0; d < W; ++d) {
            int64_t so = 0, ro = 0;
            for (int j = 0; j < d; ++j) so += counts[(size_t)s][(size_t)j];
            for (int j = 0; j < s; ++j) ro += counts[(size_t)j][(size_t)d];
            if (counts[(size_t)s][(size_t)d] > 0) plan.push_back({s, d, so, ro, counts[(size_t)s][(size_t)d]});
        }
    return plan;
}

gs_status exchange(gs_group* g, std::vector<int64_t>* nrec) {
    const int W = g->world;
    const int64_t xb = gs_exchange_record_bytes();
    // the exchange regions (gsplat.h): each moves on its own, region k of a
    // buffer of n records starting at n x (the earlier regions' bytes)
    int32_t rb[GS_XREGIONS];
    const int nreg = gs_exchange_regions(rb);
    std::vector<std::vector<int64_t>> counts((size_t)W);
    std::vector<int64_t> sent((size_t)W, 0);
    nrec->assign((size_t)W, 0);
    for (int s = 0; s < W; ++s) {
        counts[(size_t)s] = g->r[(size_t)s].counts;
        for (int d = 0; d < W; ++d) {
            (*nrec)[(size_t)d] += counts[(size_t)s][(size_t)d];
            sent[(size_t)s] += counts[(size_t)s][(size_t)d];
        }
    }
    for (int d = 0; d < W; ++d) GG_HIP(g->r[(size_t)d].recv.reserve(g->r[(size_t)d].dev, (size_t)std::max<int64_t>((*nrec)[(size_t)d], 1) * xb));
    const std::vector<Xfer> plan = exchange_plan(counts);
    if (g->transport == GS_TRANSPORT_RCCL) GG_NCCL(g_rccl.group_start());
    int64_t pre = 0;  // bytes per record of the regions before region k
    for (int k = 0; k < nreg; pre += rb[k], ++k) {
        const int64_t b = rb[k];
        for (const Xfer& x : plan) {
            Rank &ks = g->r[(size_t)x.src], &kd = g->r[(size_t)x.dst];
            char* src = ks.send.as<char>() + pre * sent[(size_t)x.src] + x.soff * b;
            char* dst = kd.recv.as<char>() + pre * (*nrec)[(size_t)x.dst] + x.roff * b;
            if (g->transport == GS_TRANSPORT_RCCL) {
                // each transfer: a send on src's communicator, the matching recv on dst's
                GG_NCCL(g_rccl.send(src, (size_t)(x.n * b), ncclUint8, x.dst, g->comms[(size_t)x.src], ks.st));
                GG_NCCL(g_rccl.recv(dst, (size_t)(x.n * b), ncclUint8, x.src, g->comms[(size_t)x.dst], kd.st));
            } else {
                GG_HIP(hipSetDevice(kd.dev));
                GG_HIP(hipStreamWaitEvent(kd.st, ks.ev_ready, 0));
                GG_HIP(hipMemcpyPeerAsync(dst, kd.dev, src, ks.dev, (size_t)(x.n * b), kd.st));
            }
        }
    }
    if (g->transport == GS_TRANSPORT_RCCL) GG_NCCL(g_rccl.group_end());
    return GS_OK;
}

gs_status gather_bands(gs_group* g, int Wd, int Ht, float* out);

gs_status render_rows(gs_group* g, const float* V, const float* P, int Wd, int Ht, float* out) {
    const int W = g->world;
    const int64_t xb = gs_exchange_record_bytes();
    gs_status s = run_ranks(g, [&](Rank& k, int) -> gs_status {
        const size_t cap = (size_t)std::max<int64_t>(gs_point_count(k.h), 1) * (size_t)W * (size_t)xb;
        GG_HIP(k.send.reserve(k.dev, cap));
        k.counts.assign((size_t)W, 0);
        gs_status st = gs_shard_project(k.h, V, P, Wd, Ht, k.send.ptr, (int64_t)k.send.bytes, k.counts.data(), k.st);
        if (st != GS_OK) return st;
        GG_HIP(hipEventRecord(k.ev_ready, k.st));
        return GS_OK;
    });
    if (s != GS_OK) return s;
    std::vector<int64_t> nrec;
    if ((s = exchange(g, &nrec)) != GS_OK) return s;
    if ((s = run_ranks(g, [&](Rank& k, int d) -> gs_status {
             int row0, nrows;
             owned_rows(Ht, W, d, &row0, &nrows);
             GG_HIP(k.band.reserve(k.dev, (size_t)std::max(nrows, 1) * gs::kBin * Wd * 16));
             gs_status st = gs_shard_render(k.h, k.recv.ptr, nrec[(size_t)d], Wd, Ht, k.band.as<float>(), k.st);
             if (st != GS_OK) return st;
             GG_HIP(hipEventRecord(k.ev_done, k.st));
             return GS_OK;
         })) != GS_OK)
        return s;
    return gather_bands(g, Wd, Ht, out);
}

// Bands (owned rows stacked, contiguous under the default table) into the
// frame on devices[0]: RCCL send/recv straight into `out`, or peer copies.
gs_status gather_bands(gs_group* g, int Wd, int Ht, float* out) {
    const int W = g->world;
    Rank& r0 = g->r[0];
    auto span = [&](int d, size_t* off, size_t* bytes) {
        int row0, nrows;
        owned_rows(Ht, W, d, &row0, &nrows);
        const int y0 = row0 * gs::kBin, y1 = std::min(Ht, (row0 + nrows) * gs::kBin);
        *off = (size_t)y0 * Wd * 4;
        *bytes = y1 > y0 ? (size_t)(y1 - y0) * Wd * 16 : 0;
    };
    if (g->transport == GS_TRANSPORT_RCCL) {
        GG_NCCL(g_rccl.group_start());
        for (int d = 1; d < W; ++d) {
            size_t off, bytes;
            span(d, &off, &bytes);
            if (!bytes) continue;
            GG_NCCL(g_rccl.send(g->r[(size_t)d].band.ptr, bytes, ncclUint8, 0, g->comms[(size_t)d], g->r[(size_t)d].st));
            GG_NCCL(g_rccl.recv(out + off, bytes, ncclUint8, d, g->comms[0], r0.st));
        }
        GG_NCCL(g_rccl.group_end());
        size_t off, bytes;
        span(0, &off, &bytes);
        GG_HIP(hipSetDevice(r0.dev));
        if (bytes) GG_HIP(hipMemcpyAsync(out + off, r0.band.ptr, bytes, hipMemcpyDeviceToDevice, r0.st));
        for (int d = 1; d < W; ++d) {  // the senders' streams are done with their bands
            GG_HIP(hipSetDevice(g->r[(size_t)d].dev));
            GG_HIP(hipEventRecord(g->r[(size_t)d].ev_done, g->r[(size_t)d].st));
        }
        GG_HIP(hipSetDevice(r0.dev));
        for (int d = 1; d < W; ++d) GG_HIP(hipStreamWaitEvent(r0.st, g->r[(size_t)d].ev_done, 0));
        return GS_OK;
    }
    GG_HIP(hipSetDevice(r0.dev));
    for (int d = 0; d < W; ++d) {
        size_t off, bytes;
        span(d, &off, &bytes);
        if (!bytes) continue;
        GG_HIP(hipStreamWaitEvent(r0.st, g->r[(size_t)d].ev_done, 0));
        GG_HIP(hipMemcpyPeerAsync(out + off, r0.dev, g->r[(size_t)d].band.ptr, g->r[(size_t)d].dev, bytes, r0.st));
    }
    return GS_OK;
}

// Replicated-scene bands: each rank renders its owned rows
// of the whole scene (gs_band_render), then the band gather.
gs_status render_bands(gs_group* g, const float* V, const float* P, int Wd, int Ht, float* out) {
    gs_status s = run_ranks(g, [&](Rank& k, int d) -> gs_status {
        int row0, nrows;
        owned_rows(Ht, g->world, d, &row0, &nrows);
        GG_HIP(k.band.reserve(k.dev, (size_t)std::max(nrows, 1) * gs::kBin * Wd * 16));
        gs_status st = gs_band_render(k.h, V, P, Wd, Ht, k.band.as<float>(), k.st);
        if (st != GS_OK) return st;
        GG_HIP(hipEventRecord(k.ev_done, k.st));
        return GS_OK;
    });
    if (s != GS_OK) return s;
    return gather_bands(g, Wd, Ht, out);
}

gs_status render_slabs(gs_group* g, const float* V, const float* P, int Wd, int Ht, float* out) {
    const int W = g->world;
    const int64_t xb = gs_exchange_record_bytes();
    const size_t npx = (size_t)Wd * Ht;
    gs_status s = run_ranks(g, [&](Rank& k, int) -> gs_status {
        GG_HIP(k.hist.reserve(k.dev, GS_SLAB_BINS * 8));
        gs_status st = gs_slab_project(k.h, V, P, Wd, Ht, k.hist.as<uint64_t>(), k.st);
        if (st != GS_OK) return st;
        GG_HIP(hipEventRecord(k.ev_ready, k.st));
        return GS_OK;
    });
    if (s != GS_OK) return s;
    // histogram all-reduce -> the same slab bounds on every rank
    std::vector<uint64_t> hsum(GS_SLAB_BINS, 0), hk(GS_SLAB_BINS);
    if (g->transport == GS_TRANSPORT_RCCL) {
        GG_NCCL(g_rccl.group_start());
        for (int i = 0; i < W; ++i)
            GG_NCCL(g_rccl.all_reduce(g->r[(size_t)i].hist.ptr, g->r[(size_t)i].hist.ptr, GS_SLAB_BINS, ncclUint64, ncclSum,
                                      g->comms[(size_t)i], g->r[(size_t)i].st));
        GG_NCCL(g_rccl.group_end());
        GG_HIP(hipSetDevice(g->r[0].dev));
        GG_HIP(hipMemcpyAsync(hsum.data(), g->r[0].hist.ptr, GS_SLAB_BINS * 8, hipMemcpyDeviceToHost, g->r[0].st));
        GG_HIP(hipEventRecord(g->r[0].ev_ready, g->r[0].st));
        if ((s = wait_bounded(g, g->r[0].dev, g->r[0].ev_ready, "slab histogram all-reduce")) != GS_OK) return s;
    } else {
        for (int i = 0; i < W; ++i) {
            GG_HIP(hipSetDevice(g->r[(size_t)i].dev));
            GG_HIP(hipMemcpyAsync(hk.data(), g->r[(size_t)i].hist.ptr, GS_SLAB_BINS * 8, hipMemcpyDeviceToHost,
                                  g->r[(size_t)i].st));
            GG_HIP(hipStreamSynchronize(g->r[(size_t)i].st));
            for (int b = 0; b < GS_SLAB_BINS; ++b) hsum[(size_t)b] += hk[(size_t)b];
        }
    }
    std::vector<uint32_t> bounds((size_t)W + 1);
    if ((s = gs_slab_bounds(hsum.data(), W, bounds.data())) != GS_OK) return s;
    if ((s = run_ranks(g, [&](Rank& k, int) -> gs_status {
             const size_t cap = (size_t)std::max<int64_t>(gs_point_count(k.h), 1) * (size_t)xb;
             GG_HIP(k.send.reserve(k.dev, cap));
             k.counts.assign((size_t)W, 0);
             gs_status st = gs_slab_pack(k.h, bounds.data(), k.send.ptr, (int64_t)k.send.bytes, k.counts.data(), k.st);
             if (st != GS_OK) return st;
             GG_HIP(hipEventRecord(k.ev_ready, k.st));
             return GS_OK;
         })) != GS_OK)
        return s;
    std::vector<int64_t> nrec;
    if ((s = exchange(g, &nrec)) != GS_OK) return s;
    if ((s = run_ranks(g, [&](Rank& k, int d) -> gs_status {
             GG_HIP(k.tloc.reserve(k.dev, npx * 4));
             GG_HIP(k.tall.reserve(k.dev, npx * 4 * (size_t)W));
             GG_HIP(k.contrib.reserve(k.dev, npx * 16));
             gs_status st = gs_slab_render(k.h, k.recv.ptr, nrec[(size_t)d], Wd, Ht, k.tloc.as<float>(), k.st);
             if (st != GS_OK) return st;
             GG_HIP(hipEventRecord(k.ev_ready, k.st));
             return GS_OK;
         })) != GS_OK)
        return s;
    // all-gather of the slabs' transmittance, rank-major
    if (g->transport == GS_TRANSPORT_RCCL) {
        GG_NCCL(g_rccl.group_start());
        for (int i = 0; i < W; ++i)
            GG_NCCL(g_rccl.all_gather(g->r[(size_t)i].tloc.ptr, g->r[(size_t)i].tall.ptr, npx, ncclFloat32,
                                      g->comms[(size_t)i], g->r[(size_t)i].st));
        GG_NCCL(g_rccl.group_end());
    } else {
        for (int d = 0; d < W; ++d) {
            Rank& k = g->r[(size_t)d];
            GG_HIP(hipSetDevice(k.dev));
            for (int j = 0; j < W; ++j) {
                GG_HIP(hipStreamWaitEvent(k.st, g->r[(size_t)j].ev_ready, 0));
                GG_HIP(hipMemcpyPeerAsync(k.tall.as<float>() + (size_t)j * npx, k.dev, g->r[(size_t)j].tloc.ptr,
                                          g->r[(size_t)j].dev, npx * 4, k.st));
            }
        }
    }
    if ((s = run_ranks(g, [&](Rank& k, int) -> gs_status {
             gs_status st = gs_slab_composite(k.h, k.tall.as<float>(), k.contrib.as<float>(), k.st);
             if (st != GS_OK) return st;
             GG_HIP(hipEventRecord(k.ev_done, k.st));
             return GS_OK;
         })) != GS_OK)
        return s;
    // RGBA + weight reduce (SUM) into the frame on devices[0]
    Rank& r0 = g->r[0];
    if (g->transport == GS_TRANSPORT_RCCL) {
        GG_NCCL(g_rccl.group_start());
        for (int i = 0; i < W; ++i)
            GG_NCCL(g_rccl.reduce(g->r[(size_t)i].contrib.ptr, i == 0 ? (void*)out : g->r[(size_t)i].contrib.ptr,
                                  npx * 4, ncclFloat32, ncclSum, 0, g->comms[(size_t)i], g->r[(size_t)i].st));
        GG_NCCL(g_rccl.group_end());
        for (int d = 1; d < W; ++d) {
            GG_HIP(hipSetDevice(g->r[(size_t)d].dev));
            GG_HIP(hipEventRecord(g->r[(size_t)d].ev_done, g->r[(size_t)d].st));
        }
        GG_HIP(hipSetDevice(r0.dev));
        for (int d = 1; d < W; ++d) GG_HIP(hipStreamWaitEvent(r0.st, g->r[(size_t)d].ev_done, 0));
        return GS_OK;
    }
    // rank order: frame = c0, frame += c1, ... (the virtual-slab reference's order)
    GG_HIP(hipSetDevice(r0.dev));
    GG_HIP(r0.stage.reserve(r0.dev, npx * 16));
    GG_HIP(hipMemcpyAsync(out, r0.contrib.ptr, npx * 16, hipMemcpyDeviceToDevice, r0.st));
    for (int d = 1; d < W; ++d) {
        GG_HIP(hipStreamWaitEvent(r0.st, g->r[(size_t)d].ev_done, 0));
        GG_HIP(hipMemcpyPeerAsync(r0.stage.ptr, r0.dev, g->r[(size_t)d].contrib.ptr, g->r[(size_t)d].dev, npx * 16,
                                  r0.st));
        GG_HIP(gs::launch_accumulate(reinterpret_cast<float4*>(out), r0.stage.as<const float4>(), npx, r0.st));
    }
    return GS_OK;
}

// ---- two frames in flight, rows scheme (gs_group_render_pipelined) ---------

#ifndef GS_GROUP_SPLIT  // A/B knob: 1 = a pipelined rank render's composite on the rank's gather stream
#define GS_GROUP_SPLIT 1
#endif

// The ranks' compute / exchange / gather streams and their events, and (RCCL)
// a second communicator set for the all-to-all, so that frame k's exchange
// and frame k-1's gather, issued on different streams, never share a
// communicator.  Made at the first pipelined frame.
gs_status ensure_pipeline(gs_group* g) {
    if (g->pipe_ready) return GS_OK;
    for (Rank& k : g->r) {
        GG_HIP(hipSetDevice(k.dev));
        for (hipStream_t* q : {&k.cs, &k.xs, &k.gs})
            if (!*q) GG_HIP(hipStreamCreateWithFlags(q, hipStreamNonBlocking));
        for (hipEvent_t* e : {&k.ev_proj, &k.ev_xdone[0], &k.ev_xdone[1], &k.ev_rdone[0], &k.ev_rdone[1], &k.ev_gdone})
            if (!*e) GG_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
        // (recorded once, so every first wait on them is satisfied at once)
        for (hipEvent_t e : {k.ev_xdone[0], k.ev_xdone[1], k.ev_rdone[0], k.ev_rdone[1], k.ev_gdone})
            GG_HIP(hipEventRecord(e, k.cs));
    }
    if (g->transport == GS_TRANSPORT_RCCL && g->xcomms.empty()) {
        std::vector<int> dev;
        for (const Rank& k : g->r) dev.push_back(k.dev);
        g->xcomms.assign((size_t)g->world, nullptr);
        const ncclResult_t rc = g_rccl.comm_init_all(g->xcomms.data(), g->world, dev.data());
        if (rc != ncclSuccess) {
            g->xcomms.clear();
            return gfail(GS_ERR_COMM, std::string("ncclCommInitAll (exchange communicators): ") + g_rccl.error_string(rc));
        }
    }
    g->pipe_ready = true;
    return GS_OK;
}

// Frame k's all-to-all from slot s's send buffers into slot s's receive
// buffers, on the exchange streams: each waits for its rank's projection of
// frame k and for the render that last read its receive buffer (frame k-2).
// The same transfer plan as exchange(), so the copy transport the one-GPU
// tests run checks the offsets the RCCL path uses.
gs_status exchange_pipelined(gs_group* g, int s, std::vector<int64_t>* nrec) {
    const int W = g->world;
    const int64_t xb = gs_exchange_record_bytes();
    int32_t rb[GS_XREGIONS];
    const int nreg = gs_exchange_regions(rb);
    std::vector<std::vector<int64_t>> counts((size_t)W);
    std::vector<int64_t> sent((size_t)W, 0);
    nrec->assign((size_t)W, 0);
    for (int q = 0; q < W; ++q) {
        counts[(size_t)q] = g->r[(size_t)q].pcounts[s];
        for (int d = 0; d < W; ++d) {
            (*nrec)[(size_t)d] += counts[(size_t)q][(size_t)d];
            sent[(size_t)q] += counts[(size_t)q][(size_t)d];
        }
    }
    for (int d = 0; d < W; ++d) {
        Rank& kd = g->r[(size_t)d];
        GG_HIP(hipSetDevice(kd.dev));
        const size_t want = (size_t)std::max<int64_t>((*nrec)[(size_t)d], 1) * xb;
        if (want > kd.precv[s].bytes) GG_HIP(hipEventSynchronize(kd.ev_rdone[s]));  // (growth frees the buffer)
        GG_HIP(kd.precv[s].reserve(kd.dev, want));
        GG_HIP(hipStreamWaitEvent(kd.xs, kd.ev_rdone[s], 0));
        for (const Rank& ks : g->r) GG_HIP(hipStreamWaitEvent(kd.xs, ks.ev_proj, 0));  // (every source's records)
    }
    const std::vector<Xfer> plan = exchange_plan(counts);
    if (g->transport == GS_TRANSPORT_RCCL) GG_NCCL(g_rccl.group_start());
    int64_t pre = 0;
    for (int k = 0; k < nreg; pre += rb[k], ++k) {
        const int64_t b = rb[k];
        for (const Xfer& x : plan) {
            Rank &ks = g->r[(size_t)x.src], &kd = g->r[(size_t)x.dst];
            char* src = ks.psend[s].as<char>() + pre * sent[(size_t)x.src] + x.soff * b;
            char* dst = kd.precv[s].as<char>() + pre * (*nrec)[(size_t)x.dst] + x.roff * b;
            if (g->transport == GS_TRANSPORT_RCCL) {
                GG_NCCL(g_rccl.send(src, (size_t)(x.n * b), ncclUint8, x.dst, g->xcomms[(size_t)x.src], ks.xs));
                GG_NCCL(g_rccl.recv(dst, (size_t)(x.n * b), ncclUint8, x.src, g->xcomms[(size_t)x.dst], kd.xs));
            } else {
                GG_HIP(hipSetDevice(kd.dev));
                GG_HIP(hipMemcpyPeerAsync(dst, kd.dev, src, ks.dev, (size_t)(x.n * b), kd.xs));
            }
        }
    }
    if (g->transport == GS_TRANSPORT_RCCL) GG_NCCL(g_rccl.group_end());
    for (Rank& k : g->r) {
        GG_HIP(hipSetDevice(k.dev));
        GG_HIP(hipEventRecord(k.ev_xdone[s], k.xs));
    }
    return GS_OK;
}

// The rendered frame's bands into `out` on the gather streams (each waits for
// its rank's render), then the caller's stream waits for the gather.
gs_status gather_pipelined(gs_group* g, int Wd, int Ht, float* out, hipStream_t user) {
    const int W = g->world;
    Rank& r0 = g->r[0];
    auto span = [&](int d, size_t* off, size_t* bytes) {
        int row0, nrows;
        owned_rows(Ht, W, d, &row0, &nrows);
        const int y0 = row0 * gs::kBin, y1 = std::min(Ht, (row0 + nrows) * gs::kBin);
        *off = (size_t)y0 * Wd * 4;
        *bytes = y1 > y0 ? (size_t)(y1 - y0) * Wd * 16 : 0;
    };
    for (Rank& k : g->r) {
        GG_HIP(hipSetDevice(k.dev));
        GG_HIP(hipStreamWaitEvent(k.gs, k.ev_done, 0));
    }
    GG_HIP(hipSetDevice(r0.dev));
    for (int d = 1; d < W; ++d) GG_HIP(hipStreamWaitEvent(r0.gs, g->r[(size_t)d].ev_done, 0));
    if (g->transport == GS_TRANSPORT_RCCL) {
        GG_NCCL(g_rccl.group_start());
        for (int d = 1; d < W; ++d) {
            size_t off, bytes;
            span(d, &off, &bytes);
            if (!bytes) continue;
            GG_NCCL(g_rccl.send(g->r[(size_t)d].band.ptr, bytes, ncclUint8, 0, g->comms[(size_t)d], g->r[(size_t)d].gs));
            GG_NCCL(g_rccl.recv(out + off, bytes, ncclUint8, d, g->comms[0], r0.gs));
        }
        GG_NCCL(g_rccl.group_end());
    } else {
        GG_HIP(hipSetDevice(r0.dev));
        for (int d = 1; d < W; ++d) {
            size_t off, bytes;
            span(d, &off, &bytes);
            if (bytes)
                GG_HIP(hipMemcpyPeerAsync(out + off, r0.dev, g->r[(size_t)d].band.ptr, g->r[(size_t)d].dev, bytes, r0.gs));
        }
    }
    size_t off, bytes;
    span(0, &off, &bytes);
    GG_HIP(hipSetDevice(r0.dev));
    if (bytes) GG_HIP(hipMemcpyAsync(out + off, r0.band.ptr, bytes, hipMemcpyDeviceToDevice, r0.gs));
    for (Rank& k : g->r) {  // (each band is free again once its transfer is done)
        GG_HIP(hipSetDevice(k.dev));
        GG_HIP(hipEventRecord(k.ev_gdone, k.gs));
    }
    GG_HIP(hipSetDevice(r0.dev));
    GG_HIP(hipStreamWaitEvent(user, r0.ev_gdone, 0));
    return GS_OK;
}

// One pipelined call: (project) frame k and its all-to-all; the frame in
// flight (k-1) rendered and gathered into `out` (*produced = 1).  flush:
// project = false.
gs_status render_rows_pipelined(gs_group* g, const float* V, const float* P, int Wd, int Ht, float* out,
                                hipStream_t user, bool project, bool* produced) {
    *produced = false;
    gs_status st = ensure_pipeline(g);
    if (st != GS_OK) return st;
    const int W = g->world;
    const int s = g->pslot;
    const int64_t xb = gs_exchange_record_bytes();
    const gs_group::Pending prev = g->pend;
    // (bounded host waits, SURVEY §5: frame k-2's all-to-all, whose send
    // buffers this projection reuses; an RCCL peer error or a hang fails the
    // call here instead of stalling a stream sync below)
    for (Rank& k : g->r)
        if ((st = wait_bounded(g, k.dev, k.ev_xdone[s], "pipelined all-to-all")) != GS_OK) return st;
    // 1. per rank, on its compute stream: frame k's projection and packing
    //    (the host reads its destination counts), then frame k-1's render
    st = run_ranks(g, [&](Rank& k, int d) -> gs_status {
        if (project) {
            // (slot s's send buffers were last read by frame k-2's all-to-all)
            for (const Rank& o : g->r) GG_HIP(hipStreamWaitEvent(k.cs, o.ev_xdone[s], 0));
            const size_t cap = (size_t)std::max<int64_t>(gs_point_count(k.h), 1) * (size_t)W * (size_t)xb;
            if (cap > k.psend[s].bytes) GG_HIP(hipStreamSynchronize(k.cs));
            GG_HIP(k.psend[s].reserve(k.dev, cap));
            k.pcounts[s].assign((size_t)W, 0);
            gs_status r = gs_shard_project(k.h, V, P, Wd, Ht, k.psend[s].ptr, (int64_t)k.psend[s].bytes,
                                           k.pcounts[s].data(), k.cs);
            if (r != GS_OK) return r;
            GG_HIP(hipEventRecord(k.ev_proj, k.cs));
        }
        if (prev.on) {
            // the previous frame's records (its all-to-all) and a free band
            // (the gather before it, possibly read by rank 0's gather stream)
            GG_HIP(hipStreamWaitEvent(k.cs, k.ev_xdone[prev.slot], 0));
            GG_HIP(hipStreamWaitEvent(k.cs, k.ev_gdone, 0));
            GG_HIP(hipStreamWaitEvent(k.cs, g->r[0].ev_gdone, 0));
            int row0, nrows;
            owned_rows(prev.height, W, d, &row0, &nrows);
            const size_t bb = (size_t)std::max(nrows, 1) * gs::kBin * prev.width * 16;
            if (bb > k.band.bytes) {
                GG_HIP(hipEventSynchronize(k.ev_gdone));
                GG_HIP(hipEventSynchronize(g->r[0].ev_gdone));
            }
            GG_HIP(k.band.reserve(k.dev, bb));
            // (GS_GROUP_SPLIT: the render's composite on the rank's gather
            // stream, after its last gather and before the next, so the next
            // projection on the compute stream runs beside it)
            const hipStream_t cq = GS_GROUP_SPLIT ? k.gs : k.cs;
            gs_status r = GS_GROUP_SPLIT ? gs_shard_render_split(k.h, k.precv[prev.slot].ptr, prev.nrec[(size_t)d],
                                                                 prev.width, prev.height, k.band.as<float>(), k.cs, k.gs)
                                         : gs_shard_render(k.h, k.precv[prev.slot].ptr, prev.nrec[(size_t)d],
                                                           prev.width, prev.height, k.band.as<float>(), k.cs);
            if (r != GS_OK) return r;
            GG_HIP(hipEventRecord(k.ev_rdone[prev.slot], cq));
            GG_HIP(hipEventRecord(k.ev_done, cq));
        }
        return GS_OK;
    });
    if (st != GS_OK) return st;
    // (frame k-2's gather, which frame k-1's render queued behind: bounded)
    for (Rank& k : g->r)
        if ((st = wait_bounded(g, k.dev, k.ev_gdone, "pipelined gather")) != GS_OK) return st;
    // 2. frame k's all-to-all on the exchange streams, under frame k-1's render
    g->pend.on = false;
    if (project) {
        if ((st = exchange_pipelined(g, s, &g->pend.nrec)) != GS_OK) return st;
        g->pend.on = true;
        g->pend.slot = s;
        g->pend.width = Wd;
        g->pend.height = Ht;
        g->pslot = s ^ 1;
    }
    // 3. frame k-1's bands into the frame, on the gather streams
    if (prev.on) {
        if ((st = gather_pipelined(g, prev.width, prev.height, out, user)) != GS_OK) return st;
        *produced = true;
    }
    return GS_OK;
}

gs_status make_group(gs_handle* scene, int32_t num_gpus, gs_group** out, bool replicated = false) {
    if (num_gpus < 1 || num_gpus > gs::kMaxWorld) return gfail(GS_ERR_INVALID_ARG, "num_gpus must be 1..32");
    gs_group* g = new gs_group();
    g->world = num_gpus;
    g->n = gs_point_count(scene);
    g->replicated = replicated;
    g->scheme = replicated ? GS_SCHEME_BANDS : GS_SCHEME_ROWS;
    g->r.resize((size_t)num_gpus);
    for (int i = 0; i < num_gpus; ++i) {
        Rank& k = g->r[(size_t)i];
        k.dev = -1;
        k.base = replicated ? 0 : g->n * i / num_gpus;
        const int64_t e = replicated ? g->n : g->n * (i + 1) / num_gpus;
        gs_status s = gs_create_subset(scene, k.base, e, &k.h);
        if (s == GS_OK) s = gs_shard_configure(k.h, i, num_gpus, k.base);
        if (s != GS_OK) {
            delete g;
            return s;
        }
    }
    *out = g;
    return GS_OK;
}

}  // namespace

extern "C" {

gs_status gs_create_sharded_from_handle(const gs_handle* scene, int32_t num_gpus, gs_group** out) {
    if (!out || !scene) return gfail(GS_ERR_INVALID_ARG, "null argument");
    *out = nullptr;
    return make_group(const_cast<gs_handle*>(scene), num_gpus, out);
}

gs_status gs_create_replicated_from_handle(const gs_handle* scene, int32_t num_gpus, gs_group** out) {
    if (!out || !scene) return gfail(GS_ERR_INVALID_ARG, "null argument");
    *out = nullptr;
    return make_group(const_cast<gs_handle*>(scene), num_gpus, out, true);
}

gs_status gs_create_replicated(const char* ply_path, const gs_options* opt, int32_t num_gpus, gs_group** out) {
    if (!out || !ply_path) return gfail(GS_ERR_INVALID_ARG, "null argument");
    *out = nullptr;
    gs_handle* scene = nullptr;
    gs_status s = gs_create(ply_path, opt, &scene);
    if (s != GS_OK) return s;
    s = make_group(scene, num_gpus, out, true);
    gs_destroy(scene);
    return s;
}

gs_status gs_create_sharded(const char* ply_path, const gs_options* opt, int32_t num_gpus, gs_group** out) {
    if (!out || !ply_path) return gfail(GS_ERR_INVALID_ARG, "null argument");
    *out = nullptr;
    gs_handle* scene = nullptr;
    gs_status s = gs_create(ply_path, opt, &scene);
    if (s != GS_OK) return s;
    s = make_group(scene, num_gpus, out);
    gs_destroy(scene);
    return s;
}

gs_status gs_group_initialize(gs_group* g, const int32_t* devices, int32_t transport) {
    if (!g) return gfail(GS_ERR_INVALID_ARG, "null group");
    if (g->initialized) return gfail(GS_ERR_STATE, "group already initialized");
    // the environment's default wait bound, unless gs_group_set_timeout set one;
    // a value that is not a positive integer is rejected, not clamped
    if (const char* t = std::getenv("GS_COMM_TIMEOUT_MS"); t && !g->timeout_set) {
        char* end = nullptr;
        errno = 0;
        const long long v = std::strtoll(t, &end, 10);
        if (end == t || *end != '\0' || errno == ERANGE || v <= 0)
            return gfail(GS_ERR_INVALID_ARG, std::string("GS_COMM_TIMEOUT_MS is not a positive integer: '") + t + "'");
        g->timeout_ms = v;
    }
    int count = 0;
    GG_HIP(hipGetDeviceCount(&count));
    std::vector<int> dev((size_t)g->world);
    for (int i = 0; i < g->world; ++i) {
        dev[(size_t)i] = devices ? devices[i] : i;
        if (dev[(size_t)i] < 0 || dev[(size_t)i] >= count)
            return gfail(GS_ERR_DEVICE, "no HIP device " + std::to_string(dev[(size_t)i]));
    }
    std::vector<int> sorted = dev;
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    if (transport != GS_TRANSPORT_AUTO && transport != GS_TRANSPORT_RCCL && transport != GS_TRANSPORT_COPY)
        return gfail(GS_ERR_INVALID_ARG, "bad transport");
    // RCCL is loaded before any rank state exists: AUTO falls back to peer
    // copies when it cannot be loaded, an explicit RCCL request fails cleanly
    if (transport == GS_TRANSPORT_AUTO) {
        std::string why;
        transport = (distinct && g->world > 1 && g_rccl.load(&why)) ? GS_TRANSPORT_RCCL : GS_TRANSPORT_COPY;
    } else if (transport == GS_TRANSPORT_RCCL) {
        if (!distinct && !std::getenv("GS_RCCL_LIB"))
            return gfail(GS_ERR_INVALID_ARG, "RCCL needs one device per rank (GS_TRANSPORT_COPY for shared devices)");
        std::string why;
        if (!g_rccl.load(&why)) return gfail(GS_ERR_COMM, why);
        if (!distinct && !g_rccl.shared_devices)
            return gfail(GS_ERR_INVALID_ARG, "RCCL needs one device per rank (GS_TRANSPORT_COPY for shared devices)");
    }
    // Per-rank state; on failure the streams and events made here are
    // released again, so a retry starts clean (gs_initialize is idempotent
    // per handle and device).
    auto rollback = [&](gs_status st) {
        const std::string msg = gs_last_error();
        for (auto& k : g->r) {
            if (k.dev >= 0) (void)hipSetDevice(k.dev);
            if (k.own_stream && k.st) (void)hipStreamDestroy(k.st);
            if (k.ev_ready) (void)hipEventDestroy(k.ev_ready);
            if (k.ev_done) (void)hipEventDestroy(k.ev_done);
            k.st = nullptr;
            k.own_stream = false;
            k.ev_ready = k.ev_done = nullptr;
        }
        gscomm::destroy_all(g->comms, [](ncclComm_t c) { return g_rccl.comm_destroy(c); });
        return gfail(st, msg);
    };
    for (int i = 0; i < g->world; ++i) {
        Rank& k = g->r[(size_t)i];
        k.dev = dev[(size_t)i];
        gs_status s = gs_initialize(k.h, k.dev);
        hipError_t e = s == GS_OK ? hipSetDevice(k.dev) : hipSuccess;
        if (s == GS_OK && e == hipSuccess && i > 0) {
            e = hipStreamCreateWithFlags(&k.st, hipStreamNonBlocking);
            k.own_stream = e == hipSuccess;
        }
        if (s == GS_OK && e == hipSuccess) e = hipEventCreateWithFlags(&k.ev_ready, hipEventDisableTiming);
        if (s == GS_OK && e == hipSuccess) e = hipEventCreateWithFlags(&k.ev_done, hipEventDisableTiming);
        if (s == GS_OK && e != hipSuccess) {
            gs_set_last_error(std::string("gs_group_initialize: ") + hipGetErrorString(e));
            s = e == hipErrorOutOfMemory ? GS_ERR_OOM : GS_ERR_DEVICE;
        }
        if (s != GS_OK) return rollback(s);
    }
    if (transport == GS_TRANSPORT_COPY && distinct) {  // direct peer access over xGMI where the devices allow it
        for (int a = 0; a < g->world; ++a)
            for (int b = 0; b < g->world; ++b) {
                int can = 0;
                if (a == b || hipDeviceCanAccessPeer(&can, dev[(size_t)a], dev[(size_t)b]) != hipSuccess || !can) continue;
                GG_HIP(hipSetDevice(dev[(size_t)a]));
                hipError_t e = hipDeviceEnablePeerAccess(dev[(size_t)b], 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) GG_HIP(e);
                (void)hipGetLastError();
            }
    }
    if (transport == GS_TRANSPORT_RCCL) {
        g->comms.assign((size_t)g->world, nullptr);
        const ncclResult_t r = g_rccl.comm_init_all(g->comms.data(), g->world, dev.data());
        if (r != ncclSuccess) {
            gs_set_last_error(std::string("ncclCommInitAll: ") + g_rccl.error_string(r));
            return rollback(GS_ERR_COMM);
        }
    }
    if (hipSetDevice(dev[0]) != hipSuccess || hipEventCreateWithFlags(&g->frame_done, hipEventDisableTiming) != hipSuccess) {
        gs_set_last_error("gs_group_initialize: frame event");
        return rollback(GS_ERR_DEVICE);
    }
    g->transport = transport;
    g->pool = new Pool(g->world);
    g->initialized = true;
    return GS_OK;
}

gs_status gs_group_set_timeout(gs_group* g, int32_t timeout_ms) {
    if (!g || timeout_ms <= 0) return gfail(GS_ERR_INVALID_ARG, "gs_group_set_timeout: bad arguments");
    g->timeout_ms = timeout_ms;
    g->timeout_set = true;
    return GS_OK;
}

gs_status gs_group_set_scheme(gs_group* g, int32_t scheme) {
    if (!g || (scheme != GS_SCHEME_ROWS && scheme != GS_SCHEME_SLABS && scheme != GS_SCHEME_BANDS))
        return gfail(GS_ERR_INVALID_ARG, "scheme must be GS_SCHEME_ROWS, GS_SCHEME_SLABS or GS_SCHEME_BANDS");
    if ((scheme == GS_SCHEME_BANDS) != g->replicated)
        return gfail(GS_ERR_INVALID_ARG, g->replicated ? "a replicated group renders GS_SCHEME_BANDS only"
                                                       : "GS_SCHEME_BANDS needs a replicated group (gs_create_replicated)");
    g->scheme = scheme;
    return GS_OK;
}

int64_t gs_group_point_count(const gs_group* g) { return g ? g->n : 0; }
int32_t gs_group_size(const gs_group* g) { return g ? g->world : 0; }
int32_t gs_group_transport(const gs_group* g) { return g && g->initialized ? g->transport : -1; }

gs_status gs_group_set_frames_in_flight(gs_group* g, int32_t n) {
    if (!g || n < 1 || n > 2) return gfail(GS_ERR_INVALID_ARG, "gs_group_set_frames_in_flight: 1 or 2");
    if (g->pend.on) return gfail(GS_ERR_STATE, "a frame is in flight: gs_group_flush first");
    g->frames_in_flight = n;
    return GS_OK;
}

namespace {

// gs_group_render_pipelined / gs_group_flush: one call of the pipeline.
gs_status pipelined_call(gs_group* g, const float* view, const float* proj, int32_t width, int32_t height,
                         float* out_rgba, int32_t out_is_device, void* hip_stream, int32_t* produced, bool project) {
    if (!g || !g->initialized) return gfail(GS_ERR_STATE, "gs_group_initialize not called");
    if (g->failed) return gfail(GS_ERR_COMM, "group unusable after a collective failure");
    if (!produced || !out_rgba || (project && (!view || !proj || width <= 0 || height <= 0)))
        return gfail(GS_ERR_INVALID_ARG, "gs_group_render_pipelined: bad arguments");
    *produced = 0;
    if (g->frames_in_flight < 2 || g->scheme != GS_SCHEME_ROWS || g->world < 2)
        return gfail(GS_ERR_STATE, "pipelined frames: rows scheme, 2+ ranks, gs_group_set_frames_in_flight(2)");
    Rank& r0 = g->r[0];
    GG_HIP(hipSetDevice(r0.dev));
    hipStream_t user = static_cast<hipStream_t>(hip_stream);
    const int ow = g->pend.on ? g->pend.width : width, oh = g->pend.on ? g->pend.height : height;
    const size_t bytes = (size_t)ow * oh * 16;
    float* out = out_rgba;
    if (!out_is_device) {
        // (the staging frame may still be read by the last call's copy)
        GG_HIP(hipStreamSynchronize(user));
        GG_HIP(g->fb.reserve(r0.dev, bytes));
        out = g->fb.as<float>();
    }
    bool made = false;
    gs_status s = render_rows_pipelined(g, view, proj, width, height, out, user, project, &made);
    if (s != GS_OK) return s;
    *produced = made ? 1 : 0;
    GG_HIP(hipSetDevice(r0.dev));
    GG_HIP(hipEventRecord(g->frame_done, user));
    if (made && !out_is_device) {
        GG_HIP(hipMemcpyAsync(out_rgba, out, bytes, hipMemcpyDeviceToHost, user));
        GG_HIP(hipEventRecord(g->frame_done, user));
        return wait_bounded(g, r0.dev, g->frame_done, "frame");
    }
    return GS_OK;
}

}  // namespace

gs_status gs_group_render_pipelined(gs_group* g, const float* view, const float* proj, int32_t width, int32_t height,
                                    float* out_rgba, int32_t out_is_device, void* hip_stream, int32_t* produced) {
    return pipelined_call(g, view, proj, width, height, out_rgba, out_is_device, hip_stream, produced, true);
}

gs_status gs_group_flush(gs_group* g, float* out_rgba, int32_t out_is_device, void* hip_stream, int32_t* produced) {
    if (g && !g->pend.on) {  // nothing in flight
        if (!produced) return gfail(GS_ERR_INVALID_ARG, "gs_group_flush: null produced");
        *produced = 0;
        return GS_OK;
    }
    return pipelined_call(g, nullptr, nullptr, 0, 0, out_rgba, out_is_device, hip_stream, produced, false);
}

gs_status gs_group_render(gs_group* g, const float* view, const float* proj, int32_t width, int32_t height,
                          float* out_rgba, int32_t out_is_device, void* hip_stream) {
    if (!g || !g->initialized) return gfail(GS_ERR_STATE, "gs_group_initialize not called");
    if (g->failed) return gfail(GS_ERR_COMM, "group unusable after a collective failure");
    if (g->pend.on) return gfail(GS_ERR_STATE, "a pipelined frame is in flight: gs_group_flush first");
    if (!view || !proj || !out_rgba || width <= 0 || height <= 0)
        return gfail(GS_ERR_INVALID_ARG, "gs_group_render: bad arguments");
    Rank& r0 = g->r[0];
    GG_HIP(hipSetDevice(r0.dev));
    r0.st = static_cast<hipStream_t>(hip_stream);
    float* out = out_rgba;
    const size_t bytes = (size_t)width * height * 16;
    if (!out_is_device) {
        GG_HIP(g->fb.reserve(r0.dev, bytes));
        out = g->fb.as<float>();
    }
    // the last frame is done everywhere (its gather waited for every rank)
    gs_status s = wait_bounded(g, r0.dev, g->frame_done, "previous frame");
    if (s != GS_OK) return s;
    GG_HIP(hipSetDevice(r0.dev));
    s = g->world == 1 ? gs_render(r0.h, view, proj, width, height, out, 1, r0.st)
                 : g->scheme == GS_SCHEME_SLABS ? render_slabs(g, view, proj, width, height, out)
                 : g->scheme == GS_SCHEME_BANDS ? render_bands(g, view, proj, width, height, out)
                                                : render_rows(g, view, proj, width, height, out);
    if (s != GS_OK) return s;
    GG_HIP(hipSetDevice(r0.dev));
    GG_HIP(hipEventRecord(g->frame_done, r0.st));
    if (!out_is_device) {
        GG_HIP(hipMemcpyAsync(out_rgba, out, bytes, hipMemcpyDeviceToHost, r0.st));
        GG_HIP(hipEventRecord(g->frame_done, r0.st));
        return wait_bounded(g, r0.dev, g->frame_done, "frame");
    }
    // device output: asynchronous on the caller's stream (stats are read
    // lazily by gs_group_last_stats)
    return GS_OK;
}

gs_status gs_group_last_stats(gs_group* g, int32_t rank, gs_stats* out) {
    if (!g || !out || rank < 0 || rank >= g->world) return gfail(GS_ERR_INVALID_ARG, "gs_group_last_stats: bad arguments");
    return gs_last_stats(g->r[(size_t)rank].h, out);
}

void gs_group_destroy(gs_group* g) { delete g; }

}  // extern "C"
