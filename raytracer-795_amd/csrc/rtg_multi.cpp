// rtg_multi.cpp — multi-GPU fan-out of the render loop behind the C ABI.
//
// The reference parallelises inside Scene::renderScene: 8 std::threads, thread t renders the
// pixel columns x = t (mod 8) of one shared Image (src/Scene.cpp:269-292, 340-356).  Here the
// fork is over GPUs (SURVEY.md §8(b) Threading row, §8(e)): shard r of N renders every sample of
// the image rows with (y / row_block) % N == r into a compact buffer on its own device, and the
// shards' rows are gathered onto the output device with RCCL point-to-point transfers over xGMI
// (rank 0 receives N buffers of 1/N frame each, one per link, instead of a ring reduce that moves
// about twice the frame through every link).  The gather is exact: rows are copied, not summed.
// Two callers share the shard + gather code (render_shard, gather_rows):
//   * in-process (rtg_render_opts.num_devices): one host thread per device, scene replicas made by
//     device-to-device copies (scene_replicate), communicators from ncclCommInitAll;
//   * one process per GPU (rtg_comm_* + rtg_render_ranked, e.g. under torch.distributed.run):
//     communicator from ncclCommInitRank.
// RCCL is resolved at run time (dlopen of librccl.so.1): a process that already holds a
// librccl.so.1 (PyTorch's) shares it, and single-GPU users never load it.
#include <dlfcn.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <functional>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>   // types and constants only: the entry points come from dlsym

#include "../../include/rtg.h"
#include "rtg_internal.h"

namespace rtg {
namespace {

struct Rccl {
    void* handle = nullptr;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
    // non-blocking communicators (rtg_comm_init_rank_timeout): optional, the bounded waits need them
    ncclResult_t (*CommInitRankConfig)(ncclComm_t*, int, ncclUniqueId, int, ncclConfig_t*) = nullptr;
    ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;
    ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
};

std::mutex g_rccl_mu;
Rccl g_rccl;
bool g_rccl_tried = false;
std::string g_rccl_err;

int load_rccl(const Rccl** out) {
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    if (!g_rccl_tried) {
        g_rccl_tried = true;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char* e = dlerror();
            g_rccl_err = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
        } else {
            Rccl r;
            r.handle = h;
            bool ok = true;
            auto sym = [&](auto& fn, const char* name) {
                fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
                ok = ok && fn != nullptr;
            };
            sym(r.GetUniqueId, "ncclGetUniqueId");
            sym(r.CommInitRank, "ncclCommInitRank");
            sym(r.CommInitAll, "ncclCommInitAll");
            sym(r.CommDestroy, "ncclCommDestroy");
            sym(r.Send, "ncclSend");
            sym(r.Recv, "ncclRecv");
            sym(r.AllReduce, "ncclAllReduce");
            sym(r.GroupStart, "ncclGroupStart");
            sym(r.GroupEnd, "ncclGroupEnd");
            sym(r.GetErrorString, "ncclGetErrorString");
            if (ok) {
                r.CommInitRankConfig = reinterpret_cast<decltype(r.CommInitRankConfig)>(dlsym(h, "ncclCommInitRankConfig"));
                r.CommGetAsyncError = reinterpret_cast<decltype(r.CommGetAsyncError)>(dlsym(h, "ncclCommGetAsyncError"));
                r.CommAbort = reinterpret_cast<decltype(r.CommAbort)>(dlsym(h, "ncclCommAbort"));
                g_rccl = r;
            }
            else g_rccl_err = "librccl.so.1 lacks an RCCL entry point";
        }
    }
    if (!g_rccl.handle) return set_error(RTG_ERR_UNSUPPORTED, g_rccl_err);
    *out = &g_rccl;
    return RTG_OK;
}

int nccl_fail(const Rccl& R, ncclResult_t e, const char* what) {
    return set_error(RTG_ERR_HIP, std::string(what) + ": " + (R.GetErrorString ? R.GetErrorString(e) : "RCCL error"));
}

// Device buffer owned by one device.
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    int device = -1;
    int grow(int dev, size_t need) {
        if (p && device == dev && need <= bytes) return RTG_OK;
        release();
        if (hipSetDevice(dev) != hipSuccess) return set_error(RTG_ERR_NO_DEVICE, "device " + std::to_string(dev));
        if (hipMalloc(&p, need) != hipSuccess) {
            p = nullptr;
            return set_error(RTG_ERR_OOM, "hipMalloc failed (" + std::to_string(need) + " bytes)");
        }
        bytes = need;
        device = dev;
        return RTG_OK;
    }
    void release() {
        if (p) {
            int cur = 0;
            (void)hipGetDevice(&cur);
            (void)hipSetDevice(device);
            (void)hipFree(p);
            (void)hipSetDevice(cur);
        }
        p = nullptr;
        bytes = 0;
        device = -1;
    }
    float* f() const { return static_cast<float*>(p); }
};

ShardPrefix shard_prefix(int ny, int nranks, int block) {
    ShardPrefix pre{};
    for (int r = 0; r < nranks; r++) pre.rows[r + 1] = pre.rows[r] + rtg_shard_rows(ny, r, nranks, block);
    return pre;
}

// The options of shard `rank` of `nranks`: its row blocks, compact output.
rtg_render_opts shard_opts(const rtg_render_opts& o, int rank, int nranks, int block) {
    rtg_render_opts so = o;
    so.row_offset = rank;
    so.row_stride = nranks;
    so.row_block = block;
    so.compact_rows = 1;
    so.num_devices = 0;
    so.devices = nullptr;
    return so;
}

// Rank `rank` of `nranks` sends its compact rows (`part`) to rank 0; rank 0 receives every shard
// (its own through an RCCL self send/recv) into `recv`, stacked in rank order, and places the rows
// into `frame`.  Everything is enqueued on `st` (a stream of the rank's device).
// settle (non-blocking communicators): waits until the grouped transfers are enqueued on `st`, before
// anything else goes on the stream.
int gather_rows(const Rccl& R, ncclComm_t comm, int rank, int nranks, int nx, int ny, int block, const float* part,
                float* recv, float* frame, hipStream_t st, const std::function<int()>& settle = nullptr) {
    const ShardPrefix pre = shard_prefix(ny, nranks, block);
    const size_t row = (size_t)nx * 3;
    ncclResult_t e = R.GroupStart();
    if (e != ncclSuccess) return nccl_fail(R, e, "ncclGroupStart");
    if (rank == 0)
        for (int r = 0; r < nranks && e == ncclSuccess; r++) {
            const size_t n = (size_t)(pre.rows[r + 1] - pre.rows[r]) * row;
            if (n) e = R.Recv(recv + (size_t)pre.rows[r] * row, n, ncclFloat32, r, comm, st);
        }
    const size_t mine = (size_t)(pre.rows[rank + 1] - pre.rows[rank]) * row;
    if (e == ncclSuccess && mine) e = R.Send(part, mine, ncclFloat32, 0, comm, st);
    const ncclResult_t e2 = R.GroupEnd();
    if (e == ncclSuccess) e = e2;
    if (settle && e == ncclInProgress) e = ncclSuccess;
    if (e != ncclSuccess) return nccl_fail(R, e, "RCCL gather");
    if (settle)
        if (int rc = settle()) return rc;
    if (rank == 0) {
        launch_place_rows(recv, frame, nx, ny, nranks, block, pre, st);
        const hipError_t he = hipGetLastError();
        if (he != hipSuccess) return set_error(RTG_ERR_HIP, std::string("place rows: ") + hipGetErrorString(he));
    }
    return RTG_OK;
}

void add_stats(rtg_render_stats& a, const rtg_render_stats& b) {
    a.primary_rays += b.primary_rays;
    a.secondary_rays += b.secondary_rays;
    a.shadow_rays += b.shadow_rays;
    a.total_rays += b.total_rays;
    a.passes += b.passes;
    a.max_level = std::max(a.max_level, b.max_level);
    a.node_visits += b.node_visits;
    a.tri_tests += b.tri_tests;
    a.shadow_node_visits += b.shadow_node_visits;
    a.shadow_tri_tests += b.shadow_tri_tests;
    a.trace_ms += b.trace_ms;
    a.shadow_ms += b.shadow_ms;
    a.shade_ms += b.shade_ms;
    a.trace_launches += b.trace_launches;
    a.shadow_launches += b.shadow_launches;
    a.shade_launches += b.shade_launches;
    a.trace_steps += b.trace_steps;
    a.shadow_steps += b.shadow_steps;
    a.trace_lane_slots += b.trace_lane_slots;
    a.shadow_lane_slots += b.shadow_lane_slots;
    a.shadow_blocked += b.shadow_blocked;
    a.shadow_blocked_steps += b.shadow_blocked_steps;
    a.shadow_blocked_tris += b.shadow_blocked_tris;
    a.trace_entry_visits += b.trace_entry_visits;
    a.trace_entry_slots += b.trace_entry_slots;
    a.shadow_entry_visits += b.shadow_entry_visits;
    a.shadow_entry_slots += b.shadow_entry_slots;
    for (int k = 0; k < 8; k++) {
        a.shadow_hist_before[k] += b.shadow_hist_before[k];
        a.shadow_hist_after[k] += b.shadow_hist_after[k];
    }
    a.shadow_blocked_steps_before += b.shadow_blocked_steps_before;
    a.shadow_blocked_steps_before_wavemin += b.shadow_blocked_steps_before_wavemin;
    for (int k = 0; k < 4; k++) a.pt_shade_cycles[k] += b.pt_shade_cycles[k];
    for (int k = 0; k < 16; k++) {
        a.trace_entry_cycles[k] += b.trace_entry_cycles[k];
        a.shadow_entry_cycles[k] += b.shadow_entry_cycles[k];
    }
    a.resolve_ms += b.resolve_ms;
    a.accumulate_ms += b.accumulate_ms;
    a.resolve_launches += b.resolve_launches;
    a.accumulate_launches += b.accumulate_launches;
}

double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

template <class F>
int32_t guarded(F&& f) {
    try {
        return f();
    } catch (const std::bad_alloc&) {
        return set_error(RTG_ERR_OOM, "host allocation failed");
    } catch (const std::exception& e) {
        return set_error(RTG_ERR_INVALID, std::string("internal error: ") + e.what());
    }
}

}  // namespace

// Per-scene state of the in-process fan-out, kept across renders with the same device list.
struct MultiState {
    std::vector<int> devs;
    std::vector<rtg_scene*> reps;        // reps[0] = nullptr: rank 0 renders on the scene itself
    const Rccl* R = nullptr;
    std::vector<ncclComm_t> comms;       // empty when a device is listed twice (copy gather)
    std::vector<hipStream_t> streams;    // one per rank, on its device
    std::vector<DevBuf> part;            // per rank: its compact rows
    DevBuf recv;                         // on devs[0]: every shard's rows, in rank order
};

void multi_free(MultiState* m) {
    if (!m) return;
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (ncclComm_t c : m->comms)
        if (c) (void)m->R->CommDestroy(c);
    for (size_t r = 0; r < m->streams.size(); r++)
        if (m->streams[r]) {
            (void)hipSetDevice(m->devs[r]);
            (void)hipStreamDestroy(m->streams[r]);
        }
    for (rtg_scene* s : m->reps)
        if (s) rtg_scene_destroy(s);
    for (DevBuf& b : m->part) b.release();
    m->recv.release();
    delete m;
    (void)hipSetDevice(cur);
}

static int multi_setup(rtg_scene* s, const std::vector<int>& devs, MultiState** out) {
    MultiState* m = new MultiState();
    m->devs = devs;
    const int n = (int)devs.size();
    m->reps.assign(n, nullptr);
    m->streams.assign(n, nullptr);
    m->part.resize(n);
    int rc = RTG_OK;
    for (int r = 1; r < n && rc == RTG_OK; r++) rc = scene_replicate(s, devs[r], &m->reps[r]);
    for (int r = 0; r < n && rc == RTG_OK; r++) {
        if (hipSetDevice(devs[r]) != hipSuccess || hipStreamCreateWithFlags(&m->streams[r], hipStreamNonBlocking) != hipSuccess)
            rc = set_error(RTG_ERR_HIP, "stream on device " + std::to_string(devs[r]));
    }
    bool distinct = true;
    for (int a = 0; a < n; a++)
        for (int b = a + 1; b < n; b++) distinct = distinct && devs[a] != devs[b];
    if (rc == RTG_OK && distinct) {
        rc = load_rccl(&m->R);
        if (rc == RTG_OK) {
            m->comms.assign(n, nullptr);
            const ncclResult_t e = m->R->CommInitAll(m->comms.data(), n, devs.data());
            if (e != ncclSuccess) {
                m->comms.clear();
                rc = nccl_fail(*m->R, e, "ncclCommInitAll");
            }
        }
    }
    (void)hipSetDevice(scene_device(s));
    if (rc != RTG_OK) {
        multi_free(m);
        return rc;
    }
    *out = m;
    return RTG_OK;
}

int render_multi(rtg_scene* s, const rtg_camera_desc* cam, const rtg_render_opts* opts, float* out_dev, hipStream_t st) {
    const rtg_render_opts o = *opts;
    if (o.row_offset != 0 || o.row_stride > 1 || o.compact_rows)
        return set_error(RTG_ERR_INVALID, "num_devices: row_offset / row_stride / compact_rows must be 0");
    if (cam->nx < 1 || cam->ny < 1 || cam->num_samples < 1) return set_error(RTG_ERR_INVALID, "bad camera");
    int visible = 0;
    if (hipGetDeviceCount(&visible) != hipSuccess || visible < 1) return set_error(RTG_ERR_NO_DEVICE, "no HIP device");
    const int n = std::max(1, o.num_devices);
    if (n > kMaxRanks) return set_error(RTG_ERR_UNSUPPORTED, "more than 64 devices");
    const int dev0 = scene_device(s);
    std::vector<int> devs(n);
    if (o.devices) {
        for (int r = 0; r < n; r++) {
            devs[r] = o.devices[r];
            if (devs[r] < 0 || devs[r] >= visible) return set_error(RTG_ERR_NO_DEVICE, "device index out of range");
        }
        if (devs[0] != dev0) return set_error(RTG_ERR_INVALID, "devices[0] must be the scene's device");
    } else {
        if (n > visible) return set_error(RTG_ERR_NO_DEVICE, "num_devices exceeds the visible devices");
        for (int r = 0; r < n; r++) devs[r] = (dev0 + r) % visible;
    }
    if (n == 1) {
        // one device (e.g. rtg_cli --devices 1): the plain single-device render, no RCCL needed
        rtg_render_opts so = o;
        so.num_devices = 0;
        so.devices = nullptr;
        return scene_render(s, cam, &so, out_dev, st);
    }
    MultiState*& M = scene_multi(s);
    if (M && M->devs != devs) {
        multi_free(M);
        M = nullptr;
    }
    int rc;
    if (!M && (rc = multi_setup(s, devs, &M))) return rc;
    const int nx = cam->nx, ny = cam->ny;
    const int block = o.row_block > 1 ? o.row_block : 4;
    const ShardPrefix pre = shard_prefix(ny, n, block);
    for (int r = 0; r < n; r++) {
        const size_t rows = (size_t)std::max(pre.rows[r + 1] - pre.rows[r], 1);
        if ((rc = M->part[r].grow(devs[r], rows * nx * 3 * sizeof(float)))) return rc;
    }
    if ((rc = M->recv.grow(devs[0], (size_t)ny * nx * 3 * sizeof(float)))) return rc;
    (void)hipSetDevice(dev0);
    const auto t0 = std::chrono::steady_clock::now();
    // rank 0's stream starts after the work already enqueued on the caller's stream
    hipEvent_t e0 = nullptr;
    if (hipEventCreateWithFlags(&e0, hipEventDisableTiming) != hipSuccess || hipEventRecord(e0, st) != hipSuccess ||
        hipStreamWaitEvent(M->streams[0], e0, 0) != hipSuccess) {
        if (e0) (void)hipEventDestroy(e0);
        return set_error(RTG_ERR_HIP, "multi-GPU stream ordering");
    }
    (void)hipEventDestroy(e0);

    // phase 1: one host thread per device renders its shard
    std::vector<int> rcs(n, RTG_OK);
    std::vector<std::string> msgs(n);
    std::vector<rtg_render_stats> stats(n);
    auto run = [&](auto&& body) {
        std::vector<std::thread> th;
        th.reserve(n);
        for (int r = 0; r < n; r++)
            th.emplace_back([&, r] {
                rcs[r] = guarded([&]() -> int32_t {
                    if (hipSetDevice(devs[r]) != hipSuccess) return set_error(RTG_ERR_NO_DEVICE, "hipSetDevice");
                    return body(r);
                });
                if (rcs[r] != RTG_OK) msgs[r] = rtg_last_error();
            });
        for (std::thread& t : th) t.join();
        for (int r = 0; r < n; r++)
            if (rcs[r] != RTG_OK) return set_error(rcs[r], "device " + std::to_string(devs[r]) + ": " + msgs[r]);
        return (int)RTG_OK;
    };
    rc = run([&](int r) -> int32_t {
        rtg_scene* sc = r == 0 ? s : M->reps[r];
        const rtg_render_opts so = shard_opts(o, r, n, block);
        int32_t k = scene_render(sc, cam, &so, M->part[r].f(), M->streams[r]);
        if (k == RTG_OK && hipStreamSynchronize(M->streams[r]) != hipSuccess) k = set_error(RTG_ERR_HIP, "shard sync");
        stats[r] = scene_stats(sc);
        return k;
    });
    (void)hipSetDevice(dev0);
    if (rc) return rc;
    const auto t1 = std::chrono::steady_clock::now();
    // phase 2: gather the shards' rows onto devs[0]
    if (!M->comms.empty()) {
        rc = run([&](int r) -> int32_t {
            int32_t k = gather_rows(*M->R, M->comms[r], r, n, nx, ny, block, M->part[r].f(), r == 0 ? M->recv.f() : nullptr,
                                    r == 0 ? out_dev : nullptr, M->streams[r]);
            if (k == RTG_OK && hipStreamSynchronize(M->streams[r]) != hipSuccess) k = set_error(RTG_ERR_HIP, "gather sync");
            return k;
        });
        (void)hipSetDevice(dev0);
        if (rc) return rc;
    } else {
        // a device listed twice has no communicator of its own: copy the shards (rehearsal of the
        // N-shard path on fewer GPUs; the rows placed are the same)
        const size_t row = (size_t)nx * 3;
        for (int r = 0; r < n; r++) {
            const size_t bytes = (size_t)(pre.rows[r + 1] - pre.rows[r]) * row * sizeof(float);
            if (bytes && hipMemcpyPeerAsync(M->recv.f() + (size_t)pre.rows[r] * row, devs[0], M->part[r].f(), devs[r], bytes,
                                            M->streams[0]) != hipSuccess)
                return set_error(RTG_ERR_HIP, "shard copy");
        }
        launch_place_rows(M->recv.f(), out_dev, nx, ny, n, block, pre, M->streams[0]);
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(M->streams[0]) != hipSuccess)
            return set_error(RTG_ERR_HIP, "place rows");
    }
    rtg_render_stats tot{};
    for (int r = 0; r < n; r++) add_stats(tot, stats[r]);
    tot.render_ms = ms_since(t0);
    tot.gather_ms = ms_since(t1);
    tot.devices = n;
    scene_set_stats(s, tot);
    return RTG_OK;
}

}  // namespace rtg

using namespace rtg;

// One rank of a one-process-per-GPU job.  The communicator is non-blocking when the RCCL library
// has the config API (it does from NCCL 2.14 on): every wait of the rank -- set-up, the failure
// agreement, the gather -- then polls with a deadline, and a rank whose peers never join aborts the
// communicator and returns an error instead of blocking forever (`dead`: no further use).
struct rtg_comm {
    const Rccl* R = nullptr;
    ncclComm_t comm = nullptr;
    int rank = 0, nranks = 1, device = 0;
    int timeout_ms = 0;            // <= 0: no deadline (rtg_comm_init_rank)
    bool nonblocking = false;
    bool dead = false;
    DevBuf part, recv, flag;
};

namespace rtg {
namespace {
using Clock = std::chrono::steady_clock;

// The deadline of a wait that starts at t0: none (time_point::max) for a communicator set up without a
// timeout, so a peer's long shard render never aborts a healthy rank.
Clock::time_point comm_deadline(const rtg_comm* c, Clock::time_point t0) {
    return c->timeout_ms > 0 ? t0 + std::chrono::milliseconds(c->timeout_ms) : Clock::time_point::max();
}

// Wait for a non-blocking communicator's pending operation (set-up, an enqueue) to leave
// ncclInProgress, or for the deadline; on the deadline or an asynchronous error the communicator is
// aborted.  Returns RTG_OK or the error (set_error).
int comm_settle(rtg_comm* c, Clock::time_point deadline, const char* what) {
    if (!c->nonblocking) return RTG_OK;
    for (int spin = 0;; spin++) {
        ncclResult_t st = ncclSuccess;
        const ncclResult_t e = c->R->CommGetAsyncError(c->comm, &st);
        if (e != ncclSuccess) st = e;
        if (st == ncclSuccess) return RTG_OK;
        if (st != ncclInProgress) {
            (void)c->R->CommAbort(c->comm);
            c->dead = true;
            return nccl_fail(*c->R, st, what);
        }
        if (Clock::now() > deadline) {
            (void)c->R->CommAbort(c->comm);
            c->dead = true;
            return set_error(RTG_ERR_HIP, std::string(what) + ": peers did not respond within " +
                                              std::to_string(c->timeout_ms) + " ms (communicator aborted)");
        }
        if (spin < 64) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}

// Wait for the work enqueued on `st` (collectives of this communicator among it) with the same
// deadline: a peer that never posts its side of a transfer leaves the RCCL kernel spinning, so the
// stream is polled, and on the deadline the communicator is aborted (its kernels then exit).
int comm_stream_wait(rtg_comm* c, hipStream_t st, Clock::time_point deadline, const char* what) {
    if (!c->nonblocking) {
        if (hipStreamSynchronize(st) != hipSuccess) return set_error(RTG_ERR_HIP, std::string(what) + " sync");
        return RTG_OK;
    }
    for (int spin = 0;; spin++) {
        const hipError_t q = hipStreamQuery(st);
        if (q == hipSuccess) return RTG_OK;
        if (q != hipErrorNotReady) return set_error(RTG_ERR_HIP, std::string(what) + ": " + hipGetErrorString(q));
        ncclResult_t ae = ncclSuccess;
        if (c->R->CommGetAsyncError(c->comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
            (void)c->R->CommAbort(c->comm);
            c->dead = true;
            (void)hipStreamSynchronize(st);
            return nccl_fail(*c->R, ae, what);
        }
        if (Clock::now() > deadline) {
            (void)c->R->CommAbort(c->comm);
            c->dead = true;
            (void)hipStreamSynchronize(st);      // the aborted kernels return
            return set_error(RTG_ERR_HIP, std::string(what) + ": peers did not complete within " +
                                              std::to_string(c->timeout_ms) + " ms (communicator aborted)");
        }
        if (spin < 256) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
}

// Every rank learns whether any rank failed before the gather (an allreduce-sum of 0 / 1
// failure flags: the count of failed ranks), so a rank that fails early cannot leave the others
// blocked in ncclRecv / ncclSend.
// Returns the number of failed ranks seen (>= 1 means: do not gather), or < 0 when the
// agreement itself failed (the communicator is then unusable).
int agree_failures(rtg_comm* c, bool failed, hipStream_t st, Clock::time_point deadline, std::string& why) {
    if (c->flag.grow(c->device, sizeof(int32_t))) { why = "status buffer"; return -1; }
    const int32_t mine = failed ? 1 : 0;
    int32_t any = 0;
    if (hipMemcpyAsync(c->flag.p, &mine, sizeof mine, hipMemcpyHostToDevice, st) != hipSuccess) { why = "status copy"; return -1; }
    const ncclResult_t e = c->R->AllReduce(c->flag.p, c->flag.p, 1, ncclInt32, ncclSum, c->comm, st);
    if (e != ncclSuccess && !(c->nonblocking && e == ncclInProgress)) {
        why = std::string("ncclAllReduce: ") + c->R->GetErrorString(e);
        return -1;
    }
    if (comm_settle(c, deadline, "failure agreement (enqueue)") ||
        hipMemcpyAsync(&any, c->flag.p, sizeof any, hipMemcpyDeviceToHost, st) != hipSuccess ||
        comm_stream_wait(c, st, deadline, "failure agreement")) {
        why = rtg_last_error();
        return -1;
    }
    return any;
}
}  // namespace
}  // namespace rtg

extern "C" {

int32_t rtg_comm_unique_id(uint8_t id[RTG_COMM_ID_BYTES]) {
    return guarded([&]() -> int32_t {
        if (!id) return set_error(RTG_ERR_INVALID, "null id");
        static_assert(sizeof(ncclUniqueId) == RTG_COMM_ID_BYTES, "ncclUniqueId size");
        const Rccl* R = nullptr;
        int rc = load_rccl(&R);
        if (rc) return rc;
        ncclUniqueId u;
        const ncclResult_t e = R->GetUniqueId(&u);
        if (e != ncclSuccess) return nccl_fail(*R, e, "ncclGetUniqueId");
        memcpy(id, &u, sizeof u);
        return RTG_OK;
    });
}

int32_t rtg_comm_init_rank(const uint8_t id[RTG_COMM_ID_BYTES], int32_t nranks, int32_t rank, int32_t device,
                           rtg_comm** out) {
    return rtg_comm_init_rank_timeout(id, nranks, rank, device, 0, out);
}

int32_t rtg_comm_init_rank_timeout(const uint8_t id[RTG_COMM_ID_BYTES], int32_t nranks, int32_t rank, int32_t device,
                                   int32_t timeout_ms, rtg_comm** out) {
    return guarded([&]() -> int32_t {
        if (!id || !out) return set_error(RTG_ERR_INVALID, "null argument");
        *out = nullptr;
        if (nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks)
            return set_error(RTG_ERR_INVALID, "rank / nranks");
        int visible = 0;
        if (hipGetDeviceCount(&visible) != hipSuccess || device < 0 || device >= visible)
            return set_error(RTG_ERR_NO_DEVICE, "device index out of range");
        const Rccl* R = nullptr;
        int rc = load_rccl(&R);
        if (rc) return rc;
        if (hipSetDevice(device) != hipSuccess) return set_error(RTG_ERR_NO_DEVICE, "hipSetDevice");
        ncclUniqueId u;
        memcpy(&u, id, sizeof u);
        rtg_comm* k = new rtg_comm();
        k->R = R; k->rank = rank; k->nranks = nranks; k->device = device;
        k->timeout_ms = timeout_ms > 0 ? timeout_ms : 0;
        k->nonblocking = R->CommInitRankConfig && R->CommGetAsyncError && R->CommAbort;
        const auto deadline = comm_deadline(k, Clock::now());
        ncclResult_t e;
        if (k->nonblocking) {
            ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
            cfg.blocking = 0;
            e = R->CommInitRankConfig(&k->comm, nranks, u, rank, &cfg);
            if (e == ncclInProgress) e = ncclSuccess;
        } else {
            e = R->CommInitRank(&k->comm, nranks, u, rank);
        }
        if (e != ncclSuccess) {
            if (k->comm) (void)(R->CommAbort ? R->CommAbort(k->comm) : R->CommDestroy(k->comm));
            delete k;
            return nccl_fail(*R, e, "ncclCommInitRank");
        }
        if (int rc2 = comm_settle(k, deadline, "ncclCommInitRank")) {
            delete k;                            // aborted by comm_settle
            return rc2;
        }
        *out = k;
        return RTG_OK;
    });
}

int32_t rtg_comm_destroy(rtg_comm* c) {
    if (!c) return RTG_OK;
    if (c->comm && !c->dead) (void)c->R->CommDestroy(c->comm);   // an aborted communicator is freed already
    c->part.release();
    c->recv.release();
    c->flag.release();
    delete c;
    return RTG_OK;
}

int32_t rtg_render_ranked(rtg_scene* s, const rtg_camera_desc* cam, const rtg_render_opts* opts, rtg_comm* c,
                          float* frame_device, void* stream) {
    return guarded([&]() -> int32_t {
        if (!c) return set_error(RTG_ERR_INVALID, "null communicator");
        if (c->dead) return set_error(RTG_ERR_INVALID, "communicator was aborted after a timeout: destroy it");
        // The one early return that skips the failure agreement: without its device this rank
        // cannot take part in any collective, so its peers can still block in the agreement
        // until the job's own timeout (or the caller aborts the communicator).
        if (hipSetDevice(c->device) != hipSuccess) return set_error(RTG_ERR_NO_DEVICE, "hipSetDevice");
        hipStream_t st = (hipStream_t)stream;
        // Local checks and the shard render record a status instead of returning, and an
        // exception thrown by them (bad_alloc while growing a buffer, ...) becomes a status too:
        // every rank reaches the failure agreement below, whatever happened to it (no rank is
        // left waiting in the gather for a rank that gave up).
        int rc = RTG_OK;
        rtg_render_opts o{};
        if (opts) o = *opts;
        const int n = c->nranks;
        const int block = o.row_block > 1 ? o.row_block : 4;
        int nx = 0, ny = 0;
        const auto t0 = std::chrono::steady_clock::now();
        try {
            if (!s || !cam) rc = set_error(RTG_ERR_INVALID, "null argument");
            else if (c->rank == 0 && !frame_device) rc = set_error(RTG_ERR_INVALID, "rank 0 needs the frame buffer");
            else if (scene_device(s) != c->device) rc = set_error(RTG_ERR_INVALID, "scene and communicator on different devices");
            else if (cam->nx < 1 || cam->ny < 1 || cam->num_samples < 1) rc = set_error(RTG_ERR_INVALID, "bad camera");
            else if (o.num_devices > 1 || o.devices) rc = set_error(RTG_ERR_INVALID, "rtg_render_ranked: one device per rank");
            if (rc == RTG_OK) {
                nx = cam->nx;
                ny = cam->ny;
                const ShardPrefix pre = shard_prefix(ny, n, block);
                const size_t rows = (size_t)std::max(pre.rows[c->rank + 1] - pre.rows[c->rank], 1);
                rc = c->part.grow(c->device, rows * nx * 3 * sizeof(float));
                if (rc == RTG_OK && c->rank == 0) rc = c->recv.grow(c->device, (size_t)ny * nx * 3 * sizeof(float));
            }
            if (rc == RTG_OK) {
                const rtg_render_opts so = shard_opts(o, c->rank, n, block);
                rc = scene_render(s, cam, &so, c->part.f(), st);
            }
            // the shard's own completion, so the agreement + gather time below is theirs alone
            if (rc == RTG_OK && hipStreamSynchronize(st) != hipSuccess) rc = set_error(RTG_ERR_HIP, "shard render sync");
        } catch (const std::bad_alloc&) {
            rc = set_error(RTG_ERR_OOM, "host allocation failed in the shard render");
        } catch (const std::exception& e) {
            rc = set_error(RTG_ERR_HIP, std::string("shard render: ") + e.what());
        }
        const std::string local_err = rc == RTG_OK ? std::string() : std::string(rtg_last_error());
        const auto t1 = std::chrono::steady_clock::now();
        // the agreement and the gather share one deadline, counted from the shard's end
        const auto deadline = comm_deadline(c, t1);
        std::string why;
        const int failed = agree_failures(c, rc != RTG_OK, st, deadline, why);
        if (failed < 0) return set_error(RTG_ERR_HIP, "rank status agreement: " + why +
                                                         (rc != RTG_OK ? " (after: " + local_err + ")" : ""));
        if (rc != RTG_OK) return set_error(rc, local_err);
        if (failed > 0)
            return set_error(RTG_ERR_HIP, std::to_string(failed) + " other rank(s) failed before the gather");
        std::function<int()> settle;
        if (c->nonblocking) settle = [&] { return comm_settle(c, deadline, "RCCL gather (enqueue)"); };
        if ((rc = gather_rows(*c->R, c->comm, c->rank, n, nx, ny, block, c->part.f(), c->recv.f(), frame_device, st,
                              settle)))
            return rc;
        if ((rc = comm_stream_wait(c, st, deadline, "RCCL gather"))) return rc;
        rtg_render_stats t = scene_stats(s);
        t.render_ms = ms_since(t0);
        t.gather_ms = ms_since(t1);             // failure agreement + gather, after the shard finished
        t.devices = n;
        scene_set_stats(s, t);
        return RTG_OK;
    });
}

}  // extern "C"
