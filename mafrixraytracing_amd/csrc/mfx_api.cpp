// mfx_api.cpp — the extern "C" boundary (include/mafrix_rt.h).
//
// One mfx_ctx = one `Scene` on one or more GPUs. Per device the scene images live in HBM from
// mfx_create until mfx_destroy, and every render call is the wavefront pipeline's launches on
// that device's own HIP stream. A context over G devices (mfx_options.devices) is a primary
// device context plus G - 1 peers built from the same host scene; each device renders its own
// sample partition, and one RCCL reduce (a communicator the library owns, ncclCommInitAll over
// the device list) sums the FP64 accumulators into the primary's, where film and post run. No
// call falls back to a CPU path.
#include <dlfcn.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <functional>
#include <cstdlib>
#include <cstring>
#include <string>
#include <mutex>
#include <thread>
#include <vector>
#include <set>

#include "../../include/mafrix_rt.h"
#include "mfx_device.h"
#include "mfx_scene.h"
#include "mfx_wavefront.h"

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIPCHECK(expr)                                                                               \
    do {                                                                                             \
        hipError_t _e = (expr);                                                                      \
        if (_e != hipSuccess) return fail(MFX_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

// RCCL is opened when the first multi-device context is created, not linked: a process that
// already holds an RCCL (PyTorch loads its own librccl.so, soname librccl.so.1) gets that same
// instance back from dlopen by soname, so one process never maps two RCCLs; a process that
// never creates a multi-device context never loads it at all.
struct Rccl {
    decltype(&ncclCommInitAll) commInitAll = nullptr;
    decltype(&ncclCommDestroy) commDestroy = nullptr;
    decltype(&ncclReduce) reduce = nullptr;
    decltype(&ncclGroupStart) groupStart = nullptr;
    decltype(&ncclGroupEnd) groupEnd = nullptr;
    decltype(&ncclGetErrorString) errorString = nullptr;
};
const Rccl* rccl() {
    static Rccl r;
    static bool tried = false, ok = false;
    if (tried) return ok ? &r : nullptr;
    tried = true;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return nullptr;
    r.commInitAll = (decltype(r.commInitAll))dlsym(h, "ncclCommInitAll");
    r.commDestroy = (decltype(r.commDestroy))dlsym(h, "ncclCommDestroy");
    r.reduce = (decltype(r.reduce))dlsym(h, "ncclReduce");
    r.groupStart = (decltype(r.groupStart))dlsym(h, "ncclGroupStart");
    r.groupEnd = (decltype(r.groupEnd))dlsym(h, "ncclGroupEnd");
    r.errorString = (decltype(r.errorString))dlsym(h, "ncclGetErrorString");
    ok = r.commInitAll && r.commDestroy && r.reduce && r.groupStart && r.groupEnd && r.errorString;
    return ok ? &r : nullptr;
}

// IEEE binary16 bits of the half nearest x in the direction `up` (true: the least half >= x, false:
// the greatest half <= x); beyond the half range: +-inf on the outward side, +-65504 on the inward
uint16_t half_dir(float x, bool up) {
    if (std::isinf(x)) return x > 0 ? 0x7c00 : 0xfc00;
    if (x < 0) return (uint16_t)(0x8000 | half_dir(-x, !up));
    if (x == 0) return up ? 0 : 0;
    if (x > 65504.f) return up ? 0x7c00 : 0x7bff;
    int e = 0;
    (void)std::frexp((double)x, &e);  // x = m * 2^e, m in [0.5, 1)
    const int ex = std::max(e - 1, -14);  // the half's exponent (subnormals: -14)
    const double ulp = std::ldexp(1.0, ex - 10);
    const double m = (double)x / ulp;  // exact (a power-of-two scaling)
    const double k = up ? std::ceil(m) : std::floor(m);
    const double v = k * ulp;  // representable (k <= 2048)
    if (v > 65504.0) return 0x7c00;
    if (v < std::ldexp(1.0, -14)) return (uint16_t)(v / std::ldexp(1.0, -24));  // subnormal
    int ve = 0;
    const double vm = std::frexp(v, &ve);  // v = vm * 2^ve
    const int E = ve - 1;
    const int mant = (int)((vm * 2.0 - 1.0) * 1024.0);
    return (uint16_t)(((E + 15) << 10) | mant);
}
// the per-lane kernels' FP16 node: each child's box rounded outward, empty children all +inf
MfxNodeH node_to_half(const MfxNode& n) {
    MfxNodeH h;
    for (int k = 0; k < 4; ++k) {
        const bool empty = n.child[k] == MFX_CHILD_EMPTY;
        h.lox[k] = empty ? 0x7c00 : half_dir(n.lox[k], false);
        h.hix[k] = empty ? 0x7c00 : half_dir(n.hix[k], true);
        h.loy[k] = empty ? 0x7c00 : half_dir(n.loy[k], false);
        h.hiy[k] = empty ? 0x7c00 : half_dir(n.hiy[k], true);
        h.loz[k] = empty ? 0x7c00 : half_dir(n.loz[k], false);
        h.hiz[k] = empty ? 0x7c00 : half_dir(n.hiz[k], true);
        h.child[k] = n.child[k];
    }
    return h;
}

template <typename T>
hipError_t upload(T** dptr, const std::vector<T>& v) {
    size_t bytes = std::max<size_t>(sizeof(T), v.size() * sizeof(T));
    hipError_t e = hipMalloc((void**)dptr, bytes);
    if (e != hipSuccess) return e;
    if (!v.empty()) e = hipMemcpy(*dptr, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
    return e;
}
}  // namespace


// One render-ahead buffer: the RGBA8 frames that the one-sample render calls of global samples
// [base, base + n) return, the film before the first of them and the film after the last.
struct AheadBuf {
    uint8_t* frames = nullptr;          // [cap][npix][4] (y-major RGBA8)
    double* film_in = nullptr;          // [3][npix] the film before sample base (as the frames assume)
    double* film_out = nullptr;         // [3][npix] the film after sample base + n - 1
    unsigned long long* counters = nullptr;  // the batch's ray counters [WF_SHARDS][WF_NCTR]
    hipEvent_t t0 = nullptr, t1 = nullptr;   // around the batch's trace
    hipEvent_t ready = nullptr;         // frames computed
    int64_t base = 0, n = 0;            // samples held (n == 0: empty)
    int64_t expect = 0;                 // the index whose frame a call may take next
    uint64_t epoch = 0;                 // film epoch the frames were computed in
    double count0 = 0.0;                // Film frameCount before sample base
    bool reported = false;              // a call has reported the batch's rays and time
};

// k_resolve's frames mode for a wavefront trace (WfParams film / frames / count0)
struct FrameMode {
    double* film;     // the film state: read before the first sample, written after the last
    uint8_t* frames;  // null: the film only
    double count0;    // frameCount before the first sample
};

constexpr int kStageChunks = 8;  // host_readback's pipelined pieces (at most)

// mfx_sample's banded resolve (one device): the last generation's k_resolve runs in nbands column bands
// of tiles, and after each band `after(k, tx0, ntx)` enqueues that band's mean and readback, so the
// frame's copy to the host overlaps the rest of the resolve. used: wf_trace ran it (not the megakernel).
struct ResolveSplit {
    int nbands = 0;
    std::function<int(int, int, int)> after;
    bool used = false;
};

struct mfx_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    MfxHostScene host;
    MfxNode* d_nodes = nullptr;
    MfxSlot* d_slots = nullptr;
    MfxNodeH* d_nodes_h = nullptr;  // MFX_NODE_F16 builds: the FP16 copy of d_nodes (per-lane kernels)
    int32_t* d_slot_ref = nullptr;
    uint8_t* d_ref_blob = nullptr;
    MfxShade* d_shade = nullptr;
    MfxInstance* d_inst = nullptr;    // two-level scenes only
    double* d_accum = nullptr;   // [3][npix] (the active accumulator)
    double* d_accum_own = nullptr;
    double* d_film = nullptr;    // [3][npix]
    double* d_frame = nullptr;   // [npix][4] staging for x-major outputs
    uint8_t* d_rgba = nullptr;   // [npix][4]
    unsigned long long* d_work = nullptr;
    unsigned long long* d_counters = nullptr;  // [WF_SHARDS][WF_NCTR] the last trace's counters
    unsigned long long* d_counters_total = nullptr;  // [WF_SHARDS][WF_NCTR] running totals (mfx_ray_counts_total)
    uint64_t seed = 0;
    int flags = 0;
    int part_index = 0, part_count = 1;  // sample partition: global samples part_index mod part_count
    // image partition: this device traces the film's 8-pixel tile rows of band band_index of band_count
    // (band_tile_row, mfx_device.h: one of each band_count consecutive tile rows, serpentine)
    // (device g of a G-device list: g of G; an MFX_F_ROW_PARTITION rank composes with it)
    int band_index = 0, band_count = 1;
    int64_t next_sample = 0;
    double frame_count = 0.0;
    int grid = 0;
    int stack_size = 1;
    int64_t npix = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool ev_valid = false;
    // wavefront pipeline: a frame's paths run in generations of at most wf_pool_max paths
    // (mfx_wavefront.h), every iteration one bounce of every live path
    WfParams wf{};
    void* wf_mem = nullptr;
    int32_t wf_pool = 0;
    size_t wf_pool_bytes = 0;  // bytes of wf_mem
    bool wf_pool_q = false;  // the pool holds the ray queues' arrays too (allocated only for a trace that uses them)
    // MFX_RAY_QUEUE: the ray queues, and the first iteration (0-based) whose k_shadow moves the
    // continuing paths to one (-1: every iteration in place; MFX_RAY_QUEUE=0 / MFX_QUEUE_FROM=d)
    WfQueue wq[2]{};
    int wf_queue_from = MFX_RAY_QUEUE ? -2 : -1;  // -2: automatic (wf_queue_auto)
    int wf_queue_auto = 1;  // from the last trace's live paths per iteration (note_live); 1 before any
    // The first wavefront trace's counters are read once for wf_queue_auto, after every device of
    // the call has been enqueued (settle_queue_auto). Render-ahead batches settle it from each
    // batch's counters instead (note_live in ahead_render).
    bool wf_auto_read = false;
    bool wf_auto_pending = false;  // a trace whose counters settle wf_queue_auto has been enqueued
    int32_t wf_qchunk = 128;  // entries per chunk fetch on a ray queue (MFX_QCHUNK; r04j: 128 against 256, C2 8 spp +2 %)
    // Path slots of the wavefront pool, at most. A pool as large as a frame's path count (C2: 133 M
    // slots, 15 GB) runs the frame as one generation: no kernel ends with a partly filled pool
    // (+11 % on C2 over 32 M slots). Capped at 2^28 slots (31 GB of the 288 GB) and at a quarter
    // of the free HBM.
    int64_t wf_pool_max = 1 << 28;
    int64_t wf_pool_cap = 0;  // the generation cap a memory shortage left (0: none; wf_trace)
    bool pool_fail_once = false;  // MFX_POOL_FAIL_ONCE=1 (tests): the first pool allocation is refused by hipMalloc
    unsigned long long* d_wfctl = nullptr;  // [WF_CTL_ALLOC] queue 0 counts, chunk heads, queue 1 counts
    std::vector<hipEvent_t> it_ev;          // per iteration: start, extend|shadow boundary, end
    int it_recorded = 0;                    // iterations of the last trace with events in it_ev
    int it_per_gen = 0;                     // and per generation
    int generations = 0;
    bool mega_last = false;
    bool cam_last = false;  // the last wavefront trace ran its camera rays as packets (k_camera)
    int wf_ext_grid = 0, wf_shd_grid = 0;
    int wf_cam_grid = 0;  // > 0: camera rays as packets (k_camera; MFX_CAMERA_PACKETS=0 turns it off)
    int wf_chunk = 256;  // slots per chunk fetch (a multiple of 64; r04j: 256 against 1024, C2 64 spp +1 %, 8 spp +6 %)
    bool wf_shd_half = true;  // k_shadow takes half chunks in place on frames of at most 2^25 paths (MFX_SHD_HALF)
    int mega_chunk = 0;   // megakernel: paths a wave takes per atomic (0: by the call's size)
    int mega_waves = 1;   // megakernel instance: 4 (128-VGPR budget) or 1 (mfx_kernels.hip)
    int wf_stack_lds_ext = 1, wf_stack_lds_shd = 1;  // traversal stack entries per lane in LDS (the rest spill)
    int wf_ntop_ext = 0, wf_ntop_shd = 0;  // top BVH nodes each trace kernel copies into LDS
    int wf_nslot_ext = 0, wf_nslot_shd = 0;  // and slots (a small scene's whole slot array, or none)
    int wf_shadow_waves = 4;               // k_shadow's register budget: 3 or 4 waves per SIMD
    int32_t* d_spill = nullptr;      // deep traversal-stack entries
    double* d_vscratch = nullptr;    // megakernel: per-lane vertex records [max_depth + 1][6][grid * 256]
    double* d_albedo = nullptr;      // [nmat][3]
    MfxLight* d_light = nullptr;     // the light (k_shadow reads it into LDS)
    MfxCamera* d_cam = nullptr;      // the camera (k_camera reads it into LDS)
    const void** d_refs = nullptr;   // {d_slot_ref, d_ref_blob} (k_shadow reads them into LDS)
    // render-ahead (mfx_options.render_ahead; see the section above mfx_render_rgba8): one-sample
    // render calls take their frame from batches of the next render_ahead samples, traced and
    // post-processed ahead of the calls, the next batch in the background while the current one is
    // served (two buffers)
    int render_ahead = 0;
    AheadBuf ab[2];
    int ab_nbuf = 0;                 // buffers allocated (0: none yet; 1: no background batch)
    int ab_cap = 0;                  // samples per buffer
    int ab_cur = -1;                 // the buffer the last render call was served from (-1: none)
    int64_t ab_last_k = -1;          // and its index in that buffer
    uint64_t film_epoch = 1;         // bumped when the film leaves the held frames' sequence
    bool film_in_dfilm = true;       // d_film holds the film (else: ab[ab_cur].film_in + its samples up to ab_last_k)
    // d_film = ab[dfilm_buf].film_in + that batch's first dfilm_n samples (dfilm_buf >= 0): a later
    // ahead_materialize traces only the samples after those (a caller alternating
    // Render and film_mean re-traced 1, 2, ..., K - 1 samples per batch)
    int dfilm_buf = -1;
    int64_t dfilm_n = 0;
    unsigned long long* d_counters_aux = nullptr;  // ray counters of a film-only re-trace (not reported)
    hipEvent_t aux_ev0 = nullptr, aux_ev1 = nullptr;
    hipStream_t sample_copy2 = nullptr;  // mfx_sample's banded readback: a second copy stream (MFX_SAMPLE_COPY_STREAMS=2)
    hipStream_t copy_stream = nullptr;  // frame copies to the host (overlap the background trace); created
                                        // at the first render-ahead call, so a batch-only context holds one
                                        // stream (one of the process's GPU_MAX_HW_QUEUES hardware queues)
    unsigned long long* h_counters = nullptr;  // page-locked [WF_SHARDS][WF_NCTR]: a batch's ray counters
    uint8_t* h_stage = nullptr;         // page-locked staging of large readbacks (host_readback)
    hipEvent_t stage_ev[kStageChunks] = {};  // host_readback: piece i is in h_stage
    hipEvent_t band_ev[kStageChunks] = {};   // mfx_sample's banded readback: band i's mean is computed
    size_t h_stage_bytes = 0;
    bool rep_valid = false;          // the last call was served from held frames: its stats are rep_*
    double rep_counts[16] = {0};
    double rep_ms = 0.0;
    bool diag_iter = false;
    bool pooled_stream = false;  // `stream` belongs to the process's pool (process_stream), not to this context
    bool iter_events = true;  // per-iteration HIP events around each launch (mfx_trace_timing's stage split)

    // ---- multi-device (primary context only) ----
    int api_part_count = 1;              // the caller's partition count (mfx_options.part_count)
    std::vector<mfx_ctx*> peers;         // devices[1..G) of the device list, same host scene
    std::vector<ncclComm_t> comms;       // [G] one RCCL communicator per device, rank g = device g
    double* d_merge = nullptr;           // [3][npix] the devices' films merged (mfx_film_mean), allocated on first use
    bool accum_merged = true;            // the primary's accumulator holds every device's rows (mfx_accum_reduce
                                         // since the last trace or clear)
    double* d_reduce_stage = nullptr;    // repeated-device list: a peer's accumulator copied here
    std::vector<hipEvent_t> peer_done;   // repeated-device list: per peer, its trace has finished
    hipEvent_t reduce_done = nullptr;    // repeated-device list: the primary has read every peer's buffer
};

// the devices of a context, primary first
static std::vector<mfx_ctx*> devs_of(mfx_ctx* c) {
    std::vector<mfx_ctx*> v{c};
    v.insert(v.end(), c->peers.begin(), c->peers.end());
    return v;
}

// tile rows of the film in a device's band (its image partition)
static int band_rows(const mfx_ctx* d) {
    const int tr = (d->host.height + 7) / 8;
    return band_row_count(d->band_index, d->band_count, tr);
}

static void ahead_free(mfx_ctx* c) {
    for (AheadBuf& B : c->ab) {
        for (void* b : {(void*)B.frames, (void*)B.film_in, (void*)B.film_out, (void*)B.counters})
            if (b) (void)hipFree(b);
        for (hipEvent_t e : {B.t0, B.t1, B.ready})
            if (e) (void)hipEventDestroy(e);
        B = AheadBuf{};
    }
    if (c->d_counters_aux) (void)hipFree(c->d_counters_aux);
    for (hipEvent_t e : {c->aux_ev0, c->aux_ev1})
        if (e) (void)hipEventDestroy(e);
    c->d_counters_aux = nullptr;
    c->aux_ev0 = c->aux_ev1 = nullptr;
    c->ab_nbuf = 0;
    c->ab_cap = 0;
    c->ab_cur = -1;
}


static void free_ctx(mfx_ctx* c) {
    if (!c) return;
    for (ncclComm_t cm : c->comms)
        if (cm) (void)rccl()->commDestroy(cm);
    c->comms.clear();
    for (mfx_ctx* p : c->peers) free_ctx(p);
    c->peers.clear();
    (void)hipSetDevice(c->device);
    for (hipEvent_t e : c->peer_done)
        if (e) (void)hipEventDestroy(e);
    if (c->reduce_done) (void)hipEventDestroy(c->reduce_done);
    if (c->d_reduce_stage) (void)hipFree(c->d_reduce_stage);
    if (c->d_merge) (void)hipFree(c->d_merge);
    void* bufs[] = {c->d_nodes, c->d_slots, c->d_slot_ref, c->d_ref_blob, c->d_shade, c->d_inst, c->d_accum_own,
                    c->d_film, c->d_frame, c->d_rgba, c->d_work, c->d_counters, c->d_counters_total, c->wf_mem, c->d_wfctl, c->d_spill, c->d_vscratch, c->d_albedo, c->d_light, c->d_cam, (void*)c->d_refs, c->d_nodes_h};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    ahead_free(c);
    if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
    if (c->sample_copy2) (void)hipStreamDestroy(c->sample_copy2);
    if (c->h_counters) (void)hipHostFree(c->h_counters);
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    for (hipEvent_t e : c->stage_ev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->band_ev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->it_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->stream && !c->pooled_stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

extern "C" {

const char* mfx_last_error(void) { return g_err.c_str(); }
int mfx_abi_version(void) { return MFX_ABI_VERSION; }

int mfx_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// MFX_STREAM_POOL=K: contexts take their stream from K streams per device that the process creates at
// its first context and keeps, round robin, instead of creating (and at destruction releasing) one
// each. The HIP runtime maps streams onto GPU_MAX_HW_QUEUES hardware queues as it creates them; a
// context created after other streams came and went (torch's stream pools, earlier contexts) can land
// on a queue another context of its frames in flight already uses, and their launches then serialize.
// Streams created first, once, keep distinct queues for the process's life (r06k, scripts/share_queues.py).
static int stream_pool_size() {
    static const int k = getenv("MFX_STREAM_POOL") ? std::max(0, std::min(16, atoi(getenv("MFX_STREAM_POOL")))) : 0;
    return k;
}
static hipError_t process_stream(int device, int k, hipStream_t* out) {
    static std::mutex mu;
    static std::vector<std::vector<hipStream_t>> pool;
    static std::vector<unsigned> next;
    std::lock_guard<std::mutex> lock(mu);
    if ((int)pool.size() <= device) {
        pool.resize(device + 1);
        next.resize(device + 1, 0);
    }
    if (pool[device].empty()) {
        for (int i = 0; i < k; ++i) {
            hipStream_t s = nullptr;
            const hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
            if (e != hipSuccess) return e;
            pool[device].push_back(s);
        }
    }
    *out = pool[device][next[device]++ % pool[device].size()];
    return hipSuccess;
}

// Device resources of a context whose host scene, device, seed, flags and partition are set:
// stream, events, the scene images in HBM, accumulators, occupancy-derived launch shapes. On
// failure the caller frees the context (free_ctx releases whatever was allocated).
static int ctx_setup(mfx_ctx* c) {
    c->npix = (int64_t)c->host.width * c->host.height;
    c->stack_size = std::max(1, c->host.stack_entries);
    if (c->stack_size > 96) return fail(MFX_E_INVALID, "mfx_create: BVH too deep for the LDS traversal stack");
#define CK(expr)                                                                               \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess) {                                                                \
            std::string m = std::string(#expr) + ": " + hipGetErrorString(_e);                 \
            return fail(_e == hipErrorOutOfMemory ? MFX_E_NOMEM : MFX_E_DEVICE, m);            \
        }                                                                                      \
    } while (0)
    CK(hipSetDevice(c->device));
    if (const int k = stream_pool_size()) {  // MFX_STREAM_POOL (see process_stream)
        CK(process_stream(c->device, k, &c->stream));
        c->pooled_stream = true;
    } else {
        CK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    }
    CK(hipHostMalloc((void**)&c->h_counters, WF_NCTR * WF_SHARDS * sizeof(unsigned long long), hipHostMallocDefault));
    CK(hipEventCreate(&c->ev0));
    CK(hipEventCreate(&c->ev1));
    CK(upload(&c->d_nodes, c->host.nodes));
    CK(upload(&c->d_slots, c->host.slots));
    if (MFX_NODE_F16 && !getenv("MFX_NODE_F32")) {  // (MFX_NODE_F32=1: the F16 build on FP32 nodes)
        std::vector<MfxNodeH> nh(c->host.nodes.size());
        for (size_t i = 0; i < nh.size(); ++i) nh[i] = node_to_half(c->host.nodes[i]);
        CK(upload(&c->d_nodes_h, nh));
    }
    CK(upload(&c->d_slot_ref, c->host.slot_ref));
    CK(upload(&c->d_ref_blob, c->host.ref_blob));
    CK(upload(&c->d_shade, c->host.shade));
    CK(upload(&c->d_albedo, c->host.albedo));
    CK(upload(&c->d_light, std::vector<MfxLight>{c->host.light}));
    CK(upload(&c->d_cam, std::vector<MfxCamera>{c->host.camera}));
    CK(upload(&c->d_refs, std::vector<const void*>{c->d_slot_ref, c->d_ref_blob}));
    const bool inst = !c->host.inst.empty();
    const int ninst = (int)c->host.inst.size();
    if (inst) {
        CK(upload(&c->d_inst, c->host.inst));
    }
    const size_t plane = sizeof(double) * (size_t)c->npix;
    CK(hipMalloc((void**)&c->d_accum_own, 3 * plane));
    c->d_accum = c->d_accum_own;
    CK(hipMalloc((void**)&c->d_film, 3 * plane));
    CK(hipMalloc((void**)&c->d_frame, 4 * plane));
    CK(hipMalloc((void**)&c->d_rgba, 4 * (size_t)c->npix));
    CK(hipMalloc((void**)&c->d_work, 64));
    CK(hipMalloc((void**)&c->d_counters, WF_NCTR * WF_SHARDS * sizeof(unsigned long long)));
    CK(hipMalloc((void**)&c->d_counters_total, WF_NCTR * WF_SHARDS * sizeof(unsigned long long)));
    CK(hipMemset(c->d_counters_total, 0, WF_NCTR * WF_SHARDS * sizeof(unsigned long long)));
    CK(hipMalloc((void**)&c->d_wfctl, WF_CTL_ALLOC * sizeof(unsigned long long)));
    {
        size_t mfree = 0, mtotal = 0;
        if (hipMemGetInfo(&mfree, &mtotal) == hipSuccess && mfree > 0) {
            const int64_t fit =
                (int64_t)(mfree / 4 / (WF_DOUBLES_PER_SLOT(c->host.max_depth + 1) * 8 +
                                       WF_WORDS_PER_SLOT(c->host.max_depth + 1) * 4));
            c->wf_pool_max = std::max<int64_t>(1 << 20, std::min<int64_t>(c->wf_pool_max, fit));
        }
    }
    // (at most 2^28 slots: k_extend's pending entries keep a slot index in 28 bits)
    c->pool_fail_once = getenv("MFX_POOL_FAIL_ONCE") && atoi(getenv("MFX_POOL_FAIL_ONCE")) != 0;
    if (const char* pm = getenv("MFX_POOL")) c->wf_pool_max = std::max<int64_t>(2048, std::min<int64_t>(1 << 28, atoll(pm)));
    c->diag_iter = getenv("MFX_DIAG_ITER") != nullptr;
    if (const char* e = getenv("MFX_ITER_EVENTS")) c->iter_events = atoi(e) != 0 || c->diag_iter;
    if (const char* qf = getenv("MFX_QUEUE_FROM")) c->wf_queue_from = MFX_RAY_QUEUE ? std::max(-2, atoi(qf)) : -1;
    if (const char* qc = getenv("MFX_QCHUNK")) c->wf_qchunk = std::max(64, std::min(WF_CHUNK_MAX, atoi(qc) / 64 * 64));
    if (const char* rq = getenv("MFX_RAY_QUEUE")) {
        if (atoi(rq) == 0) c->wf_queue_from = -1;
    }
    if (const char* ck = getenv("MFX_MEGA_CHUNK")) c->mega_chunk = std::max(1, atoi(ck));
    // MFX_F_IN_FLIGHT: the caller alternates frames over several contexts of this device, so each
    // launch's ramp-down runs beside another frame's launches: larger chunk fetches and whole ones
    // for k_shadow (r05s, C2's 1/8 share over 3 contexts: 4.44 -> 4.37 ms, the 1/4 share 8.78 -> 8.63)
    if (c->flags & MFX_F_IN_FLIGHT) {
        c->wf_chunk = 512;
        c->wf_shd_half = false;
    }
    if (const char* e = getenv("MFX_SHD_HALF")) c->wf_shd_half = atoi(e) != 0;
    if (const char* ck = getenv("MFX_CHUNK")) {
        c->wf_chunk = std::max(64, std::min(WF_CHUNK_MAX, atoi(ck) / 64 * 64));
    }
    CK(hipMemset(c->d_accum, 0, 3 * plane));
    CK(hipMemset(c->d_film, 0, 3 * plane));
    CK(hipMemset(c->d_counters, 0, WF_NCTR * WF_SHARDS * sizeof(unsigned long long)));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, c->device));
    int bpc = 0;
    // the megakernel's register budget: 4 waves per SIMD unless the stack is deep (its spills)
    c->mega_waves = c->stack_size <= 36 ? 4 : 1;
    if (const char* e = getenv("MFX_MEGA_WAVES")) c->mega_waves = atoi(e) == 4 ? 4 : 1;
    CK(mfx_trace_occupancy(c->stack_size, &bpc, inst, c->mega_waves));
    bpc = std::max(1, std::min(bpc, 8));
    c->grid = prop.multiProcessorCount * bpc;
    // Traversal stacks, per kernel: the whole bound in LDS unless that costs resident blocks; then
    // the largest LDS share that keeps them, the deeper entries spilled to a global column (the
    // kernels' SPILL instances). Measured: with a deep BVH (C4's bound is 44 entries: k_extend 3 and
    // k_shadow 2 blocks per CU with full stacks) spilling is +14 %; where the full stacks allow
    // k_extend its 4 blocks and k_shadow 3 (C2, flat C5), k_shadow's fourth block with the largest
    // share that keeps it is +2 % (C2, C5) to +4 % (C4) (r02y: 16 entries, the round-1 rule, gained
    // nothing there).
    int ebpc = 0, sbpc = 0;
    const int shd_target_max = getenv("MFX_SHADOW_TARGET_BLOCKS") ? atoi(getenv("MFX_SHADOW_TARGET_BLOCKS")) : 8;
    for (int k = 0; k < 2; ++k) {
        const bool shd = k == 1;
        int full = 0;
        CK(mfx_wf_kernel_occupancy(shd, c->stack_size, false, 0, ninst, &full));
        int nlds = c->stack_size, blocks = full;
        if (c->stack_size > WF_STACK_LDS) {
            int b16 = 0;
            CK(mfx_wf_kernel_occupancy(shd, WF_STACK_LDS, true, 0, ninst, &b16));
            const int target = shd ? std::max(full, std::min(shd_target_max, b16)) : b16;
            if (full < target) {
                int lo = WF_STACK_LDS, hi = c->stack_size - 1;  // blocks only fall as the share grows
                while (lo < hi) {
                    const int mid = (lo + hi + 1) / 2;
                    int b = 0;
                    CK(mfx_wf_kernel_occupancy(shd, mid, true, 0, ninst, &b));
                    if (b >= target) lo = mid;
                    else hi = mid - 1;
                }
                nlds = lo;
                CK(mfx_wf_kernel_occupancy(shd, nlds, true, 0, ninst, &blocks));
            }
            if (c->diag_iter)
                fprintf(stderr, "wavefront: %s blocks/CU: full %d-entry stacks %d, %d in LDS %d; chosen %d in LDS, %d\n",
                        shd ? "k_shadow" : "k_extend", c->stack_size, full, WF_STACK_LDS, b16, nlds, blocks);
        }
        if (const char* e = getenv("MFX_STACK_LDS")) {
            nlds = std::max(1, std::min(c->stack_size, atoi(e)));
            CK(mfx_wf_kernel_occupancy(shd, nlds, nlds < c->stack_size, 0, ninst, &blocks));
        }
        (shd ? c->wf_stack_lds_shd : c->wf_stack_lds_ext) = nlds;
        (shd ? sbpc : ebpc) = blocks;
    }
    {  // top BVH nodes in LDS: as many as fit in the LDS the resident blocks leave over
        int cap = std::min((int)c->host.nodes.size(), WF_NTOP_MAX);
        if (const char* e = getenv("MFX_NTOP")) cap = std::max(0, std::min(cap, atoi(e)));
        for (int k = 0; k < 2; ++k) {
            const bool shd = k == 1;
            const int nlds = shd ? c->wf_stack_lds_shd : c->wf_stack_lds_ext, want = shd ? sbpc : ebpc;
            int lo = 0, hi = cap;  // resident blocks do not grow with ntop: bisect the largest that keeps them
            while (lo < hi) {
                const int mid = (lo + hi + 1) / 2;
                int b = 0;
                CK(mfx_wf_kernel_occupancy(shd, nlds, nlds < c->stack_size, mid, ninst, &b));
                if (b >= want) lo = mid;
                else hi = mid - 1;
            }
            (shd ? c->wf_ntop_shd : c->wf_ntop_ext) = lo;
            // A small scene's whole slot array (80-B test prefixes) in LDS too, when it fits beside the
            // top nodes without costing a resident block: every leaf test then reads LDS (C3: 26 slots)
            // (two-level scenes: none — their kernel instances never read slots from LDS)
            int ns = inst ? 0 : (int)c->host.slots.size();
            if (ns > WF_SLOT_LDS_MAX || (getenv("MFX_SLOT_LDS") && atoi(getenv("MFX_SLOT_LDS")) == 0)) ns = 0;
            if (ns > 0) {
                int b = 0;
                CK(mfx_wf_kernel_occupancy(shd, nlds, nlds < c->stack_size, lo, ninst, &b, ns));
                if (b < want) ns = 0;
            }
            (shd ? c->wf_nslot_shd : c->wf_nslot_ext) = ns;
        }
        // k_shadow with at most 3 resident blocks per CU (its LDS) runs the instance compiled for 3
        // waves per SIMD: more registers, no spills (C2 / C5 +2 %); with 4 it keeps the 4-wave one
        c->wf_shadow_waves = sbpc <= 3 ? 3 : 4;
        if (const char* e = getenv("MFX_SHADOW_WAVES")) c->wf_shadow_waves = atoi(e) == 3 ? 3 : 4;
        if (c->wf_shadow_waves == 3) sbpc = std::min(sbpc, 3);
        if (c->diag_iter)
            fprintf(stderr,
                    "wavefront: stack %d/%d (extend) %d/%d (shadow) in LDS, blocks/CU extend %d shadow %d (%d-wave "
                    "build), top nodes in LDS %d / %d, slots in LDS %d / %d\n",
                    c->wf_stack_lds_ext, c->stack_size, c->wf_stack_lds_shd, c->stack_size, ebpc, sbpc,
                    c->wf_shadow_waves, c->wf_ntop_ext, c->wf_ntop_shd, c->wf_nslot_ext, c->wf_nslot_shd);
    }
    if (const char* b = getenv("MFX_BLOCKS_PER_CU")) {  // tuning knob: resident blocks per CU (<= occupancy)
        ebpc = std::min(ebpc, std::max(1, atoi(b)));
        sbpc = std::min(sbpc, std::max(1, atoi(b)));
    }
    c->wf_ext_grid = prop.multiProcessorCount * std::max(1, std::min(ebpc, 8));
    {  // camera-ray packets (flat scenes)
        int cam = getenv("MFX_CAMERA_PACKETS") ? atoi(getenv("MFX_CAMERA_PACKETS")) : 1;
        if (cam && !inst) {
            int cb = 0;
            CK(mfx_cam_occupancy(c->stack_size, &cb));
            if (const char* e = getenv("MFX_CAM_BLOCKS")) cb = std::min(cb, std::max(1, atoi(e)));
            c->wf_cam_grid = prop.multiProcessorCount * std::max(1, std::min(cb, 8));
        }
    }
    c->wf_shd_grid = prop.multiProcessorCount * std::max(1, std::min(sbpc, 8));
    {  // deep traversal-stack entries of every lane of the larger grid
        const size_t lanes = (size_t)std::max(c->wf_ext_grid, c->wf_shd_grid) * 256;
        const int deep = c->stack_size - std::min(c->wf_stack_lds_ext, c->wf_stack_lds_shd);
        CK(hipMalloc((void**)&c->d_spill, sizeof(int32_t) * lanes * std::max(1, deep)));
    }
    CK(hipMalloc((void**)&c->d_vscratch, sizeof(double) * 6 * (size_t)(c->host.max_depth + 1) * c->grid * 256));
#undef CK
    return MFX_OK;
}

// Two-level or flat for an instanced scene. The flat image (one BVH over the expansion) is the faster
// search (C5: 5,088 vs 4,729 Mrays/s, r02bt) and exactly the same results, so it is taken whenever it
// fits the budget: traversal slots of the expansion x 512 B (slot, shade record, nodes and reference
// leaves) <= MFX_FLATTEN_MAX_BYTES (default 2 GiB; C5 is 93,698 slots, 48 MB) and, on a device,
// <= a sixteenth of its free memory. MFX_F_TWO_LEVEL keeps the instances two-level regardless;
// MFX_F_FLATTEN flattens regardless (both: rejected, MFX_E_INVALID, by the callers).
static bool flatten_instances(const mfx_scene_desc* scene, const mfx_instance* instances, int32_t ninstances,
                              int32_t flags, size_t device_free = 0) {
    if (flags & MFX_F_FLATTEN) return true;
    if (!instances || (flags & MFX_F_TWO_LEVEL)) return false;
    double budget = 2.0 * 1024 * 1024 * 1024;
    if (const char* e = getenv("MFX_FLATTEN_MAX_BYTES")) budget = atof(e);
    if (device_free > 0) budget = std::min(budget, (double)device_free / 16.0);
    double slots = 0.0;
    for (int32_t i = 0; i < ninstances; ++i) {
        const int64_t f = instances[i].first, n = instances[i].count;
        if (f < 0 || n < 0 || f + n > scene->nprims) return false;  // mfx_build_scene reports the bad entry
        for (int64_t k = f; k < f + n; ++k) slots += scene->prims[k].kind == MFX_PRIM_RECT ? 2.0 : 1.0;
    }
    return slots * 512.0 <= budget;
}

static int create_impl(const mfx_scene_desc* scene, const mfx_instance* instances, int32_t ninstances,
                       const mfx_options* opt, mfx_ctx** out) {
    if (!scene || !opt || !out) return fail(MFX_E_INVALID, "mfx_create: null argument");
    *out = nullptr;
    if (opt->part_count < 1 || opt->part_index < 0 || opt->part_index >= opt->part_count)
        return fail(MFX_E_INVALID, "mfx_create: bad sample partition");
    if (opt->ndevices < 0 || opt->ndevices > MFX_MAX_DEVICES || (opt->ndevices > 0 && !opt->devices))
        return fail(MFX_E_INVALID, "mfx_create: bad device list");
    if (opt->render_ahead < 0 || opt->render_ahead > MFX_MAX_RENDER_AHEAD)
        return fail(MFX_E_INVALID, "mfx_create: render_ahead out of range");
    if (scene->nmat > WF_MAT_MAX) return fail(MFX_E_INVALID, "mfx_create: more than 65,536 materials");
    if ((opt->flags & MFX_F_FLATTEN) && (opt->flags & MFX_F_TWO_LEVEL))
        return fail(MFX_E_INVALID, "mfx_create: MFX_F_FLATTEN and MFX_F_TWO_LEVEL exclude each other");
    int ndev = 0;
    HIPCHECK(hipGetDeviceCount(&ndev));
    std::vector<int> devlist;
    if (opt->ndevices == 0) devlist.push_back(opt->device);
    else devlist.assign(opt->devices, opt->devices + opt->ndevices);
    for (int d : devlist)
        if (d < 0 || d >= ndev) return fail(MFX_E_DEVICE, "mfx_create: no such HIP device");
    const int G = (int)devlist.size();
    HIPCHECK(hipSetDevice(devlist[0]));
    size_t dev_free = 0, dev_total = 0;
    if (hipMemGetInfo(&dev_free, &dev_total) != hipSuccess) dev_free = 0;
    mfx_ctx* c = new mfx_ctx();
    std::string err;
    // the traversal BVH is built on the first device unless the caller asks for the host build
    // (the same tree either way: tests/test_gpu_build.py); the other devices get copies
    if (!mfx_build_scene(scene, c->host, err, (opt->flags & MFX_F_HOST_BVH) == 0, instances, ninstances,
                         flatten_instances(scene, instances, ninstances, opt->flags, dev_free))) {
        delete c;
        const bool dev = err.rfind("GPU BVH build", 0) == 0;
        return fail(dev ? MFX_E_DEVICE : MFX_E_INVALID, "mfx_create: " + err);
    }
    // Image partition: device g of G traces the film's tile rows of band g of G, every sample of the
    // caller's partition, so every per-pixel operation (the sample-order sum, the film add, the post)
    // runs on one device in the one-device order: images are bit-identical to one device's, and the
    // devices' buffers merge exactly (a pixel is non-zero on its own device only). With
    // MFX_F_ROW_PARTITION the caller's part_index / part_count select tile rows too: device g renders
    // rows part_index + g * part_count of part_count * G (no sample partition).
    const bool rows = (opt->flags & MFX_F_ROW_PARTITION) != 0;
    auto init = [&](mfx_ctx* d, int g) {
        d->device = devlist[g];
        d->seed = opt->seed;
        d->flags = opt->flags;
        d->part_index = rows ? 0 : opt->part_index;
        d->part_count = rows ? 1 : opt->part_count;
        d->band_index = rows ? opt->part_index + g * opt->part_count : g;
        d->band_count = rows ? opt->part_count * G : G;
        d->api_part_count = opt->part_count;
    };
    init(c, 0);
    c->render_ahead = opt->render_ahead;
    int rc = ctx_setup(c);
    if (rc) {
        free_ctx(c);
        return rc;
    }
    if (G > 1) {  // peers: one host thread each (HIP context creation and uploads run concurrently)
        c->peers.assign(G - 1, nullptr);
        std::vector<int> prc(G - 1, MFX_OK);
        std::vector<std::string> perr(G - 1);
        std::vector<std::thread> th;
        for (int g = 1; g < G; ++g) {
            mfx_ctx* p = new mfx_ctx();
            p->host = c->host;
            init(p, g);
            c->peers[g - 1] = p;
            th.emplace_back([p, g, &prc, &perr] {
                prc[g - 1] = ctx_setup(p);
                if (prc[g - 1]) perr[g - 1] = g_err;
            });
        }
        for (auto& t : th) t.join();
        for (int g = 1; g < G; ++g)
            if (prc[g - 1]) {
                free_ctx(c);
                return fail(prc[g - 1], "device " + std::to_string(devlist[g]) + ": " + perr[g - 1]);
            }
    }
    if (opt->ndevices > 0) {
        // The device reduce. Distinct devices: one RCCL communicator per device, owned by the
        // library (ncclCommInitAll, single process). A list that repeats a device cannot form a
        // communicator: its accumulators are added into the primary's in device order instead.
        const bool distinct = std::set<int>(devlist.begin(), devlist.end()).size() == devlist.size();
        if (distinct) {
            const Rccl* R = rccl();
            if (!R) {
                free_ctx(c);
                return fail(MFX_E_DEVICE, "mfx_create: RCCL (librccl.so.1) could not be loaded");
            }
            c->comms.assign(G, nullptr);
            const ncclResult_t r = R->commInitAll(c->comms.data(), G, devlist.data());
            if (r != ncclSuccess) {
                c->comms.clear();
                free_ctx(c);
                return fail(MFX_E_DEVICE, std::string("mfx_create: ncclCommInitAll: ") + R->errorString(r));
            }
        } else {
            hipError_t e = hipSetDevice(c->device);
            if (e == hipSuccess) e = hipMalloc((void**)&c->d_reduce_stage, 3 * sizeof(double) * (size_t)c->npix);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&c->reduce_done, hipEventDisableTiming);
            for (size_t k = 0; k < c->peers.size() && e == hipSuccess; ++k) {
                hipEvent_t ev = nullptr;
                e = hipSetDevice(c->peers[k]->device);
                if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
                if (e == hipSuccess) c->peer_done.push_back(ev);
            }
            if (e == hipSuccess) e = hipSetDevice(c->device);
            if (e != hipSuccess) {
                free_ctx(c);
                return fail(MFX_E_DEVICE, std::string("mfx_create: device reduce setup: ") + hipGetErrorString(e));
            }
        }
    }
    *out = c;
    return MFX_OK;
}

int mfx_create(const mfx_scene_desc* scene, const mfx_options* opt, mfx_ctx** out) {
    return create_impl(scene, nullptr, 0, opt, out);
}

int mfx_create_instanced(const mfx_scene_desc* scene, const mfx_instance* instances, int32_t ninstances,
                         const mfx_options* opt, mfx_ctx** out) {
    if (!instances || ninstances < 1) return fail(MFX_E_INVALID, "mfx_create_instanced: no instances");
    return create_impl(scene, instances, ninstances, opt, out);
}

int mfx_expand_instances(const mfx_prim* prims, int64_t nprims, const mfx_instance* instances, int32_t ninstances,
                         mfx_prim* out, int64_t cap, int64_t* nout) {
    if (!nout) return fail(MFX_E_INVALID, "mfx_expand_instances: null count");
    std::vector<mfx_prim> w;
    std::string err;
    if (!mfx_expand(prims, nprims, instances, ninstances, w, err)) return fail(MFX_E_INVALID, "mfx_expand_instances: " + err);
    *nout = (int64_t)w.size();
    if (out) {
        if (cap < (int64_t)w.size()) return fail(MFX_E_INVALID, "mfx_expand_instances: output too small");
        std::copy(w.begin(), w.end(), out);
    }
    return MFX_OK;
}

static void instancing_info(const MfxHostScene& h, double out[8]) {
    out[0] = (double)h.inst.size();
    out[1] = h.ntemplates;
    out[2] = h.inst.empty() ? 0 : h.tlas_nodes;
    out[3] = h.blas_nodes;
    out[4] = h.blas_slots;
    out[5] = h.top_slots;
    out[6] = h.world_slots;
    out[7] = (double)(h.nodes.size() * sizeof(MfxNode) + h.slots.size() * sizeof(MfxSlot) +
                      h.inst.size() * sizeof(MfxInstance));
}

int mfx_instancing_info(mfx_ctx* c, double out[8]) {
    if (!c || !out) return fail(MFX_E_INVALID, "null argument");
    instancing_info(c->host, out);
    return MFX_OK;
}

int mfx_build_instanced_info(const mfx_scene_desc* scene, const mfx_instance* instances, int32_t ninstances,
                             int32_t flags, double out[8], int32_t* stack_entries) {
    if (!out) return fail(MFX_E_INVALID, "null argument");
    MfxHostScene h;
    std::string err;
    if (!scene) return fail(MFX_E_INVALID, "null argument");
    if ((flags & MFX_F_FLATTEN) && (flags & MFX_F_TWO_LEVEL))
        return fail(MFX_E_INVALID, "mfx_build_instanced_info: MFX_F_FLATTEN and MFX_F_TWO_LEVEL exclude each other");
    if (!mfx_build_scene(scene, h, err, false, instances, ninstances, flatten_instances(scene, instances, ninstances, flags)))
        return fail(MFX_E_INVALID, "mfx_build_instanced_info: " + err);
    instancing_info(h, out);
    if (stack_entries) *stack_entries = h.stack_entries;
    return MFX_OK;
}

void mfx_destroy(mfx_ctx* ctx) { free_ctx(ctx); }

// Allocate (or grow) the wavefront path-slot pool (SoA). queues: the trace runs ray queues
// (MFX_RAY_QUEUE), whose arrays (6 doubles and 7 words per slot) are allocated only then.
static int wf_ensure_pool(mfx_ctx* c, int32_t pool, bool queues) {
    if (pool <= c->wf_pool && (!queues || c->wf_pool_q)) return MFX_OK;
    const size_t P = (size_t)pool;
    const int nv = c->host.max_depth + 1;  // vertices per path
    const size_t per_slot = WF_DOUBLES_PER_SLOT(nv) * 8 + WF_WORDS_PER_SLOT(nv) * 4 - (queues ? 0 : WF_QUEUE_BYTES_PER_SLOT);
    const size_t bytes = P * per_slot + 64 * 256;
    // leave the runtime its headroom (kernel scratch is allocated at launch, and the runtime gives
    // an idle queue's scratch back, so a later launch allocates it again): a pool that would take
    // the device's last min(2 GiB, a quarter of what is free) counts as out of memory, and wf_trace
    // retries with smaller generations. The check runs before the current pool is freed (its bytes
    // count as free), so a refused growth keeps it: a smaller generation may fit in it.
    // It runs again after the allocation: processes sharing the device (the one-GPU rehearsal of an
    // N-rank job) that checked at the same time must not take the headroom together (r06n: eight
    // ranks' pools left no room for a launch's scratch).
    size_t mfree = 0, mtotal = 0, headroom = 0;
    if (hipMemGetInfo(&mfree, &mtotal) == hipSuccess && mfree > 0) {
        const size_t avail = mfree + (c->wf_mem ? c->wf_pool_bytes : 0);
        headroom = std::min<size_t>((size_t)2 << 30, avail / 4);
        if (bytes + headroom > avail)
            return fail(MFX_E_NOMEM, "wavefront pool: " + std::to_string(bytes >> 20) + " MiB with " +
                                         std::to_string(avail >> 20) + " MiB free");
    }
    if (c->wf_mem) (void)hipFree(c->wf_mem);
    c->wf_mem = nullptr;
    c->wf_pool = 0;
    c->wf_pool_bytes = 0;
    // (MFX_POOL_FAIL_ONCE: the first request is one the device cannot hold, as another process's
    // allocation between the check above and this one would make it)
    hipError_t e = hipMalloc(&c->wf_mem, c->pool_fail_once ? ((size_t)1 << 50) : bytes);
    c->pool_fail_once = false;
    if (e != hipSuccess) {
        // wf_trace recovers with smaller generations: clear the failure from the thread's last
        // error, or the next launch's hipGetLastError reports it as the launch's own (r06p: eight
        // ranks on one GPU failed "mfx_wf_iteration: out of memory" after a refused pool)
        (void)hipGetLastError();
        c->wf_mem = nullptr;
        return fail(e == hipErrorOutOfMemory ? MFX_E_NOMEM : MFX_E_DEVICE,
                    std::string("wavefront pool: ") + hipGetErrorString(e));
    }
    if (headroom > 0 && hipMemGetInfo(&mfree, &mtotal) == hipSuccess && mfree < headroom) {
        (void)hipFree(c->wf_mem);
        c->wf_mem = nullptr;
        return fail(MFX_E_NOMEM, "wavefront pool: " + std::to_string(bytes >> 20) + " MiB left " +
                                     std::to_string(mfree >> 20) + " MiB free");
    }
    c->wf_pool_bytes = bytes;
    char* p = (char*)c->wf_mem;
    auto take = [&](size_t n) { char* r = p; p += (n + 255) & ~(size_t)255; return r; };
    double** dbl[6] = {&c->wf.ox, &c->wf.oy, &c->wf.oz, &c->wf.dx, &c->wf.dy, &c->wf.dz};
    for (double** d : dbl) *d = (double*)take(P * 8);
    c->wf.vei = (double*)take(P * 8 * nv);
    c->wf.vls = (double*)take(P * 8 * 2 * nv);
    c->wf.vmat = (WfMat*)take(P * sizeof(WfMat) * nv);
    c->wf.vstride = (int64_t)P;
    c->wf.rn = (uint32_t*)take(P * 4);
    c->wf.depth = (int32_t*)take(P * 4);
    c->wf.state = (int32_t*)take(P * 4);
#if MFX_RAY_QUEUE
    if (queues) {
    // queue 0: its own arrays; queue 1: the pool's ray arrays (o, d, rn: dead once the
    // iterations run on queues) and its own depth, state and slot words
    WfQueue& q0 = c->wq[0];
    double** q0d[6] = {&q0.ox, &q0.oy, &q0.oz, &q0.dx, &q0.dy, &q0.dz};
    for (double** d : q0d) *d = (double*)take(P * 8);
    q0.rn = (uint32_t*)take(P * 4);
    WfQueue& q1 = c->wq[1];
    q1.ox = c->wf.ox; q1.oy = c->wf.oy; q1.oz = c->wf.oz;
    q1.dx = c->wf.dx; q1.dy = c->wf.dy; q1.dz = c->wf.dz;
    q1.rn = c->wf.rn;
    for (WfQueue* q : {&q0, &q1}) {
        q->depth = (int32_t*)take(P * 4);
        q->state = (int32_t*)take(P * 4);
        q->slot = (int32_t*)take(P * 4);
    }
    q0.count = c->d_wfctl;                                  // WF_CTL_Q0
    q1.count = c->d_wfctl - WF_CTL_Q0 + WF_CTL_Q1;
    }
#endif
    c->wf_pool = pool;
    c->wf_pool_q = queues;
    return MFX_OK;
}

// Iteration d's arrays (MFX_RAY_QUEUE, mfx_wavefront.h WfParams): the pool itself up to iteration
// q = wf_queue_from, whose k_shadow moves the continuing paths to queue 0; iteration d > q reads
// queue (d - q - 1) & 1 and writes the other. d = -1: the pool (k_resolve).
static void wf_queue_views(mfx_ctx* c, WfParams& P, int d) {
    const WfParams& A = c->wf;
    P.ox = A.ox; P.oy = A.oy; P.oz = A.oz; P.dx = A.dx; P.dy = A.dy; P.dz = A.dz;
    P.rn = A.rn; P.depth = A.depth; P.state = A.state;
    P.fstate = A.state;
    P.qslot = nullptr;
    P.qcount = nullptr;
    P.ncount = nullptr;
    const int q = c->wf_queue_from == -2 ? c->wf_queue_auto : c->wf_queue_from;
    if (q < 0 || d < 0) return;
    if (d > q) {
        const WfQueue& R = c->wq[(d - q - 1) & 1];
        P.ox = R.ox; P.oy = R.oy; P.oz = R.oz; P.dx = R.dx; P.dy = R.dy; P.dz = R.dz;
        P.rn = R.rn; P.depth = R.depth; P.state = R.state;
        P.qslot = R.slot;
        P.qcount = R.count;
    }
    if (d >= q && d < P.max_depth) {
        const WfQueue& N = c->wq[(d - q) & 1];
        P.nox = N.ox; P.noy = N.oy; P.noz = N.oz; P.ndx = N.dx; P.ndy = N.dy; P.ndz = N.dz;
        P.nrn = N.rn; P.ndepth = N.depth; P.nstate = N.state; P.nslot = N.slot;
        P.ncount = N.count;
    }
}

static void fill_scene_params(mfx_ctx* c, WfParams& P) {
    P.nodes = c->d_nodes;
#if MFX_NODE_F16
    P.nodes_h = c->d_nodes_h;
#endif
    P.slots = c->d_slots;
    P.slot_ref = c->d_slot_ref;
    P.ref_blob = c->d_ref_blob;
    P.shade = c->d_shade;
    P.inst = c->d_inst;
    P.light = c->host.light;
    P.light_dev = c->d_light;
    P.cam_dev = c->d_cam;
    P.refs_dev = c->d_refs;
    P.cam = c->host.camera;
    // a gray light (bitwise equal intensities): k_shadow records a lit vertex's direct term itself
    P.gray_light = std::memcmp(&P.light.color[0], &P.light.color[1], sizeof(double)) == 0 &&
                   std::memcmp(&P.light.color[0], &P.light.color[2], sizeof(double)) == 0 && !getenv("MFX_NO_GRAY_LIGHT");
    P.lit_in_hit = c->host.max_depth <= 3 && c->host.shade.size() <= ((size_t)1 << 25) && !getenv("MFX_NO_LIT_IN_HIT");
    P.accum = c->d_accum;
    P.albedo = c->d_albedo;
    P.nmat = (int32_t)(c->host.albedo.size() / 3);
}

static void note_live(mfx_ctx* c, const unsigned long long* h);

// The wavefront pipeline. The frame's path indices (sample-major, 8x8 tiles) are cut into
// generations of at most wf_pool_max paths; slot j of a generation holds path path_base + j. A
// generation is max_depth + 1 iterations of (k_extend, k_shadow) — the primary ray and the
// max_depth extension rays of PathIntegrator.TraceRay (Integrators.fs:107-137), one bounce of
// every live path per iteration — then k_resolve adds its finished paths to their pixels. Every
// launch count is known up front, so the whole call is enqueued without a host round trip.
// fm != null (render-ahead): the samples are one-sample render calls added to fm->film in order
// (k_resolve's frames mode), the ray counters go to `counters` and the trace is bracketed by the
// events e0 / e1 instead of the context's (no per-iteration events), so a batch traced in the
// background leaves the last call's timing records alone.
// split != null (mfx_sample, one device): the last generation's resolve in column bands (ResolveSplit).
static int wf_trace(mfx_ctx* c, int64_t ns, int64_t sample_base, const FrameMode* fm = nullptr,
                    unsigned long long* counters = nullptr, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr,
                    ResolveSplit* split = nullptr) {
    const int W = c->host.width, H = c->host.height;
    const int brows = band_rows(c);
    const int64_t per_sample = (int64_t)((W + 7) / 8) * brows * 64;  // the device's band of the film
    const int64_t total = per_sample * ns;
    if (total == 0) return fail(MFX_E_STATE, "wf_trace: empty band");
    // generations of whole 64-path windows (one 8x8 tile of one sample each: the camera-ray packets)
    const int qf = c->wf_queue_from == -2 ? c->wf_queue_auto : c->wf_queue_from;  // the ray-queue start
    int64_t gen_max = 0;
    int32_t pool = 0;
    int rc = MFX_OK;
    // the device short of memory (other contexts or processes on it): smaller generations, the same
    // images (a generation only bounds how many paths are in flight). The shrunk cap is kept, and a
    // later call goes back to the configured maximum once the device has room for twice that pool
    // (a one-off spike no longer shrinks a context for good; the margin keeps contexts of
    // several processes sharing a device from growing back into each other's launches, r06j)
    int64_t cap = c->wf_pool_cap > 0 ? c->wf_pool_cap : c->wf_pool_max;
    if (cap < c->wf_pool_max) {
        const int nv = c->host.max_depth + 1;
        const double full = (double)std::min<int64_t>(total, c->wf_pool_max) *
                            (WF_DOUBLES_PER_SLOT(nv) * 8 + WF_WORDS_PER_SLOT(nv) * 4);
        size_t mfree = 0, mtotal = 0;
        if (hipMemGetInfo(&mfree, &mtotal) == hipSuccess && 2.0 * full < (double)(mfree + c->wf_pool_bytes))
            cap = c->wf_pool_max;
    }
    while (true) {
        gen_max = std::min<int64_t>(total, std::max<int64_t>(4096, cap / 4096 * 4096));
        pool = (int32_t)((gen_max + 4095) / 4096 * 4096);  // 64 shards of whole windows
        rc = wf_ensure_pool(c, pool, qf >= 0);
        if (rc != MFX_E_NOMEM || cap <= (1 << 20)) break;
        cap = std::max<int64_t>(1 << 20, gen_max / 2);
    }
    if (rc) return rc;
    c->wf_pool_cap = cap < c->wf_pool_max ? cap : 0;
    WfParams P = c->wf;
    fill_scene_params(c, P);
    P.ctl = c->d_wfctl - WF_CTL_Q0;
    P.counters = counters ? counters : c->d_counters;
    const bool own_events = e0 == nullptr;
    // per-iteration stage events (mfx_trace_timing's split): off with MFX_ITER_EVENTS=0 (A/B of their cost)
    const bool iter_events = own_events && c->iter_events;
    P.seed = c->seed;
    P.sample_base = sample_base;
    P.part_index = c->part_index;
    P.part_count = c->part_count;
    P.band_index = c->band_index;
    P.band_count = c->band_count;
    P.band_rows = brows;
    P.width = W;
    P.height = H;
    P.max_depth = c->host.max_depth;
    P.stack_size = c->stack_size;
    P.stack_lds_ext = c->wf_stack_lds_ext;
    P.stack_lds_shd = c->wf_stack_lds_shd;
    P.ntop_ext = c->wf_ntop_ext;
    P.ntop_shd = c->wf_ntop_shd;
    P.nslot_ext = c->wf_nslot_ext;
    P.nslot_shd = c->wf_nslot_shd;
    P.shadow_waves = c->wf_shadow_waves;
    P.ninst_lds = std::min<int>((int)c->host.inst.size(), WF_INST_LDS);
    P.spill = c->d_spill;
    // slots per chunk fetch: 256 at every frame size. Round 3 used 1024 (512 for frames of at most
    // 2^25 paths); with the shard counters on lines of their own and the closed-shard mask the chunk
    // fetches no longer convoy, so small chunks cut the launches' tails (r04j: C2 fixed cost per
    // frame 1.67 -> 1.24 ms, 8 spp +8 %, 64 spp +1 %)
    P.chunk = c->wf_chunk;
    P.tile_padding = (W % 8 != 0 || H % 8 != 0) ? 1 : 0;
    const int32_t chunk0 = P.chunk;
    P.film = fm ? fm->film : nullptr;
    P.frames = fm ? fm->frames : nullptr;
    P.count0 = fm ? fm->count0 : 0.0;
    const bool stats = (c->flags & MFX_F_COUNT_STATS) != 0;
    P.cam_grid = c->host.inst.empty() ? c->wf_cam_grid : 0;
    if (own_events) c->cam_last = P.cam_grid > 0;
    const int64_t ngen = (total + gen_max - 1) / gen_max;
    const int per_gen = P.max_depth + 1;  // bounce-synchronous iterations per generation
    const int iters = (int)ngen * per_gen;
    while (iter_events && (int)c->it_ev.size() < 3 * iters) {
        hipEvent_t e;
        HIPCHECK(hipEventCreate(&e));
        c->it_ev.push_back(e);
    }
    // MFX_DIAG_ITER=1: per-iteration ray counts and stage times on stderr
    auto diag = [&](int64_t g, const char* what, int d, float fe, float fs) -> int {
        HIPCHECK(hipStreamSynchronize(c->stream));
        unsigned long long h[WF_NCTR * WF_SHARDS];
        HIPCHECK(hipMemcpy(h, c->d_counters, sizeof(h), hipMemcpyDeviceToHost));
        double r[WF_NCTR] = {0};
        for (int k = 0; k < WF_SHARDS; ++k)
            for (int q = 0; q < WF_NCTR; ++q) r[q] += (double)h[WF_NCTR * k + q];
        for (int q = WF_CTR_ITER + 1; q < WF_CTR_ITER + WF_ITER_CTRS; ++q) r[1] += r[q];
        fprintf(stderr, "gen %lld %s %d: cumulative primary %.0f ext %.0f shadow %.0f; extend %.3f ms shadow %.3f ms;"
                " stamps %.4g %.4g %.4g %.4g outer %.4g node %.4g; cumulative traversal closest %.0f %.0f %.0f"
                " shadow %.0f %.0f %.0f; scan %.4g shade %.4g lat %.4g\n", (long long)g, what, d,
                r[0], r[1], r[2], fe, fs, r[10], r[11], r[12], r[13], r[14], r[15], r[4], r[5], r[6], r[7], r[8], r[9],
                r[16], r[17], r[3]);
        return MFX_OK;
    };
    HIPCHECK(hipEventRecord(own_events ? c->ev0 : e0, c->stream));
    int it = 0;
    for (int64_t g = 0; g < ngen; ++g) {
        P.path_base = g * gen_max;
        P.base_smp = P.path_base / per_sample;
        P.base_q = P.path_base % per_sample;
        P.total = std::min<int64_t>(gen_max, total - P.path_base);
        P.pool = (int32_t)((P.total + 4095) / 4096 * 4096);
        HIPCHECK(hipMemsetAsync(P.state, 0, sizeof(int32_t) * (size_t)P.pool, c->stream));
        for (int d = 0; d < per_gen; ++d, ++it) {
            P.start = d == 0 ? 1 : 0;
            P.iter = d;
            wf_queue_views(c, P, d);
            // a queue's entries are all live rays: smaller chunks keep the launch's tail short
            P.chunk = P.qcount ? c->wf_qchunk : chunk0;
            // in place on a small frame (the strong-scaling shares), k_shadow takes half chunks: the
            // first vertex's last chunks are its launch's tail (r04u: C2 at 8 spp +2.4 %; at 64 spp
            // the same halving costs 1.5 %, so frames of more than 2^25 paths keep whole chunks)
            P.chunk_shd = (c->wf_shd_half && !P.qcount && total <= ((int64_t)1 << 25)) ? std::max(64, P.chunk / 2) : P.chunk;
            if (!iter_events) {
                HIPCHECK(mfx_wf_iteration(P, c->wf_ext_grid, c->wf_shd_grid, stats, c->stream, nullptr));
                continue;
            }
            hipEvent_t* ev = c->it_ev.data() + 3 * it;
            HIPCHECK(hipEventRecord(ev[0], c->stream));
            HIPCHECK(mfx_wf_iteration(P, c->wf_ext_grid, c->wf_shd_grid, stats, c->stream, ev + 1));
            HIPCHECK(hipEventRecord(ev[2], c->stream));
            if (c->diag_iter) {
                HIPCHECK(hipStreamSynchronize(c->stream));
                float fe = 0.f, fs = 0.f;
                HIPCHECK(hipEventElapsedTime(&fe, ev[0], ev[1]));
                HIPCHECK(hipEventElapsedTime(&fs, ev[1], ev[2]));
                const int rc = diag(g, "iter", d + 1, fe, fs);
                if (rc) return rc;
            }
        }
        wf_queue_views(c, P, -1);  // k_resolve reads the pool's final state and depth words
        if (split && g == ngen - 1) {
            // a pixel's sum is its own thread's whatever the launch: the same bits as one launch
            const int tiles_x = (W + 7) / 8;
            for (int k = 0; k < split->nbands; ++k) {
                const int tx0 = (int)((int64_t)k * tiles_x / split->nbands);
                const int tx1 = (int)((int64_t)(k + 1) * tiles_x / split->nbands);
                P.res_tx0 = tx0;
                P.res_ntx = tx1 - tx0;
                if (P.res_ntx > 0) HIPCHECK(mfx_wf_resolve(P, c->stream));
                const int rc = split->after(k, tx0, tx1 - tx0);
                if (rc) return rc;
            }
            P.res_tx0 = P.res_ntx = 0;
            split->used = true;
        } else {
            HIPCHECK(mfx_wf_resolve(P, c->stream));
        }
    }
    if (!own_events) {
        HIPCHECK(hipEventRecord(e1, c->stream));
        return MFX_OK;
    }
    HIPCHECK(hipEventRecord(c->ev1, c->stream));
    c->ev_valid = true;
    // The automatic queue start is taken from a trace's per-iteration counters: read once, after
    // the context's first wavefront trace (settle_queue_auto, once every device has been
    // enqueued), so a caller that never polls the counters gets the same kernels as one that does
    if (c->wf_queue_from == -2 && !c->wf_auto_read) c->wf_auto_pending = true;
    c->it_recorded = iter_events ? iters : 0;
    c->it_per_gen = per_gen;
    c->generations = (int)ngen;
    return MFX_OK;
}

// one device's share of mfx_trace_accumulate (its sample partition), enqueued on its stream
static int dev_trace_accumulate(mfx_ctx* c, int32_t spp, int64_t sample_base, ResolveSplit* split = nullptr) {
    HIPCHECK(hipSetDevice(c->device));
    int64_t ns = spp > c->part_index ? (spp - c->part_index + c->part_count - 1) / c->part_count : 0;
    if (band_rows(c) == 0) ns = 0;  // a film too small to give this device a tile row
    HIPCHECK(hipMemsetAsync(c->d_work, 0, 64, c->stream));
    HIPCHECK(hipMemsetAsync(c->d_counters, 0, WF_NCTR * WF_SHARDS * sizeof(unsigned long long), c->stream));
    // One sample per pixel on this device (Scene.Render's call): the megakernel, unless the caller
    // pins the wavefront. With one path per pixel its FP64 atomic add onto the zeroed accumulator
    // is exact, and its per-path arithmetic is the wavefront's, so the bits are the same; it does
    // not pay the wavefront's per-bounce launches over a 2 M-path frame (r02e: 1.7 vs 7.9 ms at 1080p).
    c->mega_last = (c->flags & MFX_F_MEGAKERNEL) != 0 || (ns == 1 && (c->flags & MFX_F_WAVEFRONT) == 0);
    if (ns == 0) {  // this partition has no sample in the call: zero rays in zero device time
        HIPCHECK(hipEventRecord(c->ev0, c->stream));
        HIPCHECK(hipEventRecord(c->ev1, c->stream));
        c->ev_valid = true;
        c->it_recorded = 0;
        c->generations = 0;
        return MFX_OK;
    }
    if (!c->mega_last) {
        const int rc = wf_trace(c, ns, sample_base, nullptr, nullptr, nullptr, nullptr, split);
        if (rc) return rc;
        HIPCHECK(mfx_launch_counters_add(c->d_counters_total, c->d_counters, WF_NCTR * WF_SHARDS, c->stream));
        return MFX_OK;
    }
    TraceParams P;
    std::memset(&P, 0, sizeof(P));
    P.nodes = c->d_nodes;
    P.slots = c->d_slots;
    P.slot_ref = c->d_slot_ref;
    P.ref_blob = c->d_ref_blob;
    P.shade = c->d_shade;
    P.inst = c->d_inst;
    P.accum = c->d_accum;
    P.work_counter = c->d_work;
    P.counters = c->d_counters;
    P.light = c->host.light;
    P.cam = c->host.camera;
    P.seed = c->seed;
    P.sample_base = sample_base;
    P.nsamples = ns;
    P.part_index = c->part_index;
    P.part_count = c->part_count;
    P.band_index = c->band_index;
    P.band_count = c->band_count;
    P.band_rows = band_rows(c);
    P.width = c->host.width;
    P.height = c->host.height;
    P.max_depth = c->host.max_depth;
    P.stack_size = c->stack_size;
    P.vscratch = c->d_vscratch;
    P.waves = c->mega_waves;
    // paths per chunk: 256, halved while fewer than 16 chunks per wave remain (a 1-spp frame:
    // 64, one path per lane per fetch; r02g/r02i A/B at 1 spp: 256 -> 64 is +21 %)
    if (c->mega_chunk > 0) {
        P.chunk = c->mega_chunk;
    } else {
        const int64_t total = (int64_t)((c->host.width + 7) / 8) * band_rows(c) * 64 * ns;
        int64_t ch = 256;
        while (ch > 64 && total / ch < 16 * (int64_t)c->grid * 4) ch /= 2;
        P.chunk = (int)ch;
    }
    HIPCHECK(hipEventRecord(c->ev0, c->stream));
    HIPCHECK(mfx_launch_trace(P, (c->flags & MFX_F_COUNT_STATS) != 0, c->grid, c->stream));
    HIPCHECK(hipEventRecord(c->ev1, c->stream));
    c->ev_valid = true;
    HIPCHECK(mfx_launch_counters_add(c->d_counters_total, c->d_counters, WF_NCTR * WF_SHARDS, c->stream));
    return MFX_OK;
}

// wf_queue_auto from the first wavefront trace's counters, read once every device of the call has
// been enqueued (a blocking read inside the per-device loop ran device 0 to completion before the
// next device was enqueued)
static int settle_queue_auto(mfx_ctx* c) {
    for (mfx_ctx* d : devs_of(c)) {
        if (!d->wf_auto_pending) continue;
        HIPCHECK(hipSetDevice(d->device));
        HIPCHECK(hipMemcpyAsync(d->h_counters, d->d_counters, WF_NCTR * WF_SHARDS * sizeof(unsigned long long),
                                hipMemcpyDeviceToHost, d->stream));
        HIPCHECK(hipStreamSynchronize(d->stream));
        note_live(d, d->h_counters);
        d->wf_auto_pending = false;
        d->wf_auto_read = true;
    }
    HIPCHECK(hipSetDevice(c->device));
    return MFX_OK;
}

// Every device enqueues its band on its own stream; nothing here waits for a device (bar the
// one-time settle_queue_auto read), so the G devices render concurrently.
int mfx_trace_accumulate(mfx_ctx* c, int32_t spp, int64_t sample_base) {
    if (!c) return fail(MFX_E_STATE, "null context");
    if (spp < 1) return fail(MFX_E_INVALID, "spp must be >= 1");
    c->rep_valid = false;  // the stats now describe this trace
    c->accum_merged = false;
    for (mfx_ctx* d : devs_of(c)) {
        const int rc = dev_trace_accumulate(d, spp, sample_base);
        if (rc) return rc;
    }
    HIPCHECK(hipSetDevice(c->device));  // the primary stays current for what the caller enqueues next
    return settle_queue_auto(c);
}

// Sum every device's accumulator into the primary's, stream-ordered after each device's trace, and
// every peer's later work (a clear or trace of its accumulator) after the reduce: the RCCL reduce
// runs on each device's own stream; the repeated-device copies run on the primary's stream, so
// each peer's stream waits for them (reduce_done) before anything the caller enqueues next.
// The devices' [3][npix] buffers buf(d) summed into dst on the primary (dst may be buf(primary)).
// A device's buffer is +0.0 outside its band (image partition), so the sum is an exact merge.
static int reduce_planes(mfx_ctx* c, double* (*buf)(mfx_ctx*), double* dst, const char* what) {
    if (!c->comms.empty()) {  // RCCL: rank g sends device g's buffer, the root reduces into dst
        const Rccl* R = rccl();  // loaded: the communicators exist
        const size_t count = 3 * (size_t)c->npix;
        const std::vector<mfx_ctx*> ds = devs_of(c);
        ncclResult_t r = R->groupStart();
        for (size_t g = 0; g < ds.size() && r == ncclSuccess; ++g) {
            HIPCHECK(hipSetDevice(ds[g]->device));
            double* src = buf(ds[g]);
            r = R->reduce(src, g == 0 ? dst : src, count, ncclFloat64, ncclSum, 0, c->comms[g], ds[g]->stream);
        }
        const ncclResult_t r2 = R->groupEnd();
        if (r == ncclSuccess) r = r2;
        if (r != ncclSuccess) return fail(MFX_E_DEVICE, std::string(what) + ": " + R->errorString(r));
        HIPCHECK(hipSetDevice(c->device));
        return MFX_OK;
    }
    // a repeated-device list: add the peers' buffers in device order (a0 + a1) + a2 ...
    const size_t bytes = 3 * sizeof(double) * (size_t)c->npix;
    HIPCHECK(hipSetDevice(c->device));
    if (dst != buf(c)) HIPCHECK(hipMemcpyAsync(dst, buf(c), bytes, hipMemcpyDeviceToDevice, c->stream));
    for (size_t k = 0; k < c->peers.size(); ++k) {
        mfx_ctx* p = c->peers[k];
        HIPCHECK(hipSetDevice(p->device));
        HIPCHECK(hipEventRecord(c->peer_done[k], p->stream));
        HIPCHECK(hipSetDevice(c->device));
        HIPCHECK(hipStreamWaitEvent(c->stream, c->peer_done[k], 0));
        HIPCHECK(hipMemcpyAsync(c->d_reduce_stage, buf(p), bytes, hipMemcpyDefault, c->stream));
        HIPCHECK(mfx_launch_accum_add(dst, c->d_reduce_stage, 3 * c->npix, c->stream));
    }
    if (!c->peers.empty()) {
        HIPCHECK(hipSetDevice(c->device));
        HIPCHECK(hipEventRecord(c->reduce_done, c->stream));
        for (mfx_ctx* p : c->peers) {
            HIPCHECK(hipSetDevice(p->device));
            HIPCHECK(hipStreamWaitEvent(p->stream, c->reduce_done, 0));
        }
        HIPCHECK(hipSetDevice(c->device));
    }
    return MFX_OK;
}

int mfx_accum_reduce(mfx_ctx* c) {
    if (!c) return fail(MFX_E_STATE, "null context");
    if (c->peers.empty() && c->comms.empty()) return MFX_OK;
    if (c->accum_merged) return MFX_OK;  // merged since the last trace or clear: a second sum would add the peers twice
    const int rc = reduce_planes(c, [](mfx_ctx* d) { return d->d_accum; }, c->d_accum, "mfx_accum_reduce");
    if (rc == MFX_OK) c->accum_merged = true;
    return rc;
}

int mfx_trace_timing(mfx_ctx* c, double out[8]) {
    if (!c || !out) return fail(MFX_E_INVALID, "null argument");
    if (c->rep_valid) {  // a call served from held frames: its batch's device time, no stage split
        for (int k = 0; k < 8; ++k) out[k] = 0.0;
        out[0] = c->rep_ms;
        return MFX_OK;
    }
    double total = 0;
    int rc = mfx_last_trace_ms(c, &total);
    if (rc) return rc;
    for (int k = 0; k < 8; ++k) out[k] = 0.0;
    out[0] = total;
    if (c->mega_last) {
        out[2] = total;
        out[5] = 1;
        out[6] = 1;
    } else {
        // [2] the closest-hit kernels (k_camera + k_extend), [4] k_shadow (+ memset), summed over
        // iterations; [1] of [2] the k_camera launches (each generation's first iteration when
        // camera rays run as packets), [3] their count; the resolve launches make up the rest of [0]
        const int per_gen = std::max(1, c->it_per_gen);
        for (int it = 0; it < c->it_recorded; ++it) {
            const hipEvent_t* ev = c->it_ev.data() + 3 * it;
            float fe = 0.f, fs = 0.f;
            HIPCHECK(hipEventElapsedTime(&fe, ev[0], ev[1]));
            HIPCHECK(hipEventElapsedTime(&fs, ev[1], ev[2]));
            out[2] += fe;
            out[4] += fs;
            if (c->cam_last && it % per_gen == 0) {
                out[1] += fe;
                out[3] += 1;
            }
        }
        out[5] = c->it_recorded;
        out[6] = c->it_recorded;
        out[7] = c->generations;
    }
    return MFX_OK;
}

int mfx_last_trace_ms(mfx_ctx* c, double* ms) {
    if (!c || !ms) return fail(MFX_E_INVALID, "null argument");
    if (c->rep_valid) {
        *ms = c->rep_ms;
        return MFX_OK;
    }
    double worst = 0.0;  // the devices run concurrently: the slowest one's time
    for (mfx_ctx* d : devs_of(c)) {
        if (!d->ev_valid) return fail(MFX_E_STATE, "no trace launch recorded yet");
        HIPCHECK(hipSetDevice(d->device));
        HIPCHECK(hipEventSynchronize(d->ev1));
        float f = 0.f;
        HIPCHECK(hipEventElapsedTime(&f, d->ev0, d->ev1));
        worst = std::max(worst, (double)f);
    }
    *ms = worst;
    return MFX_OK;
}

int mfx_accum_clear(mfx_ctx* c) {
    if (!c) return fail(MFX_E_STATE, "null context");
    c->accum_merged = false;
    for (mfx_ctx* d : devs_of(c)) {
        HIPCHECK(hipSetDevice(d->device));
        HIPCHECK(hipMemsetAsync(d->d_accum, 0, 3 * sizeof(double) * (size_t)d->npix, d->stream));
    }
    return MFX_OK;
}

int mfx_accum_device_ptr(mfx_ctx* c, void** dptr, int64_t* nbytes) {
    if (!c || !dptr || !nbytes) return fail(MFX_E_INVALID, "null argument");
    *dptr = c->d_accum;
    *nbytes = 3 * (int64_t)sizeof(double) * c->npix;
    return MFX_OK;
}

int mfx_accum_attach(mfx_ctx* c, void* dptr, int64_t nbytes) {
    if (!c) return fail(MFX_E_STATE, "null context");
    if (!dptr) {
        c->d_accum = c->d_accum_own;
        return MFX_OK;
    }
    if (nbytes < 3 * (int64_t)sizeof(double) * c->npix) return fail(MFX_E_INVALID, "attached accumulator too small");
    c->d_accum = (double*)dptr;
    c->accum_merged = false;
    return MFX_OK;
}

// Device -> caller's (pageable) host memory. A pageable destination is slow for large copies
// (mfx_sample's 66 MB FP64 frame at 1080p: ~10 ms, r03b), so a large readback goes to a page-locked
// staging buffer by DMA, in pieces, and from there to the caller's buffer by host threads, each
// copying its slice of every piece as soon as that piece has landed: the copy trails the DMA by one
// piece. r06a (scripts/readback_probe.py): the DMA alone moves 66 MB in 1.17 ms, one thread copies
// it on in 2.07 ms; 4 pieces copied by threads spawned per piece took 2.56 ms with the mean kernel.

// the page-locked staging buffer, at least `bytes` (false: none could be allocated)
static bool ensure_stage(mfx_ctx* c, size_t bytes) {
    if (bytes > c->h_stage_bytes) {
        if (c->h_stage) (void)hipHostFree(c->h_stage);
        c->h_stage = nullptr;
        c->h_stage_bytes = 0;
        if (hipHostMalloc((void**)&c->h_stage, bytes, hipHostMallocDefault) == hipSuccess) c->h_stage_bytes = bytes;
        else (void)hipGetLastError();
    }
    return c->h_stage != nullptr;
}

// Pieces [off[i], off[i] + len[i]) of h_stage, each complete once stage_ev[i] has fired, copied to
// dst at the same offsets by nt host threads (MFX_READBACK_THREADS; thread t takes slice t of every
// piece, in piece order). Returns when every piece is in dst.
static double host_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
// MFX_SAMPLE_TIMING=1 (diagnostics): the host's clock at each piece's arrival and copy, on stderr
static bool sample_timing() {
    static const bool on = getenv("MFX_SAMPLE_TIMING") && atoi(getenv("MFX_SAMPLE_TIMING")) != 0;
    return on;
}

// NUMA node of the page holding `p` (-1: unknown), by get_mempolicy(MPOL_F_NODE | MPOL_F_ADDR)
static int page_node(const void* p) {
    int node = -1;
    if (syscall(SYS_get_mempolicy, &node, nullptr, 0UL, p, 3UL) != 0) return -1;
    return node;
}
// the device's NUMA node from sysfs (-1: unknown)
static int device_node(int device) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) return -1;
    for (char* q = bus; *q; ++q) *q = (char)tolower(*q);
    const std::string path = std::string("/sys/bus/pci/devices/") + bus + "/numa_node";
    FILE* f = fopen(path.c_str(), "r");
    if (!f) return -1;
    int n = -1;
    if (fscanf(f, "%d", &n) != 1) n = -1;
    fclose(f);
    return n;
}

// rgb: the staging buffer holds interleaved RGB (24 B a pixel; off / len in its bytes, whole pixels)
// and dst RGBA (32 B a pixel): each pixel is widened with alpha 1.0 as it is copied (mfx_sample)
static int copy_staged(mfx_ctx* c, void* dst, const size_t* off, const size_t* len, int npiece, bool rgb = false) {
    int nt = 8;
    if (const char* e = getenv("MFX_READBACK_THREADS")) nt = std::max(1, std::min(32, atoi(e)));
    const bool tm = sample_timing();
    double t_ready[kStageChunks] = {0}, t_copied[kStageChunks] = {0};
    const double t0 = tm ? host_ms() : 0.0;
    auto work = [&](int t) -> hipError_t {
        for (int i = 0; i < npiece; ++i) {
            const hipError_t e = hipEventSynchronize(c->stage_ev[i]);
            if (e != hipSuccess) return e;
            if (tm && t == 0) t_ready[i] = host_ms();
            if (rgb) {
                const size_t npx = len[i] / 24, p0 = off[i] / 24;
                const size_t part = (npx / nt + 63) & ~(size_t)63;  // whole pixels, 64 at a time
                if (part * t >= npx) continue;
                const double* src = (const double*)c->h_stage + 3 * (p0 + part * t);
                double* out = (double*)dst + 4 * (p0 + part * t);
                const size_t n = std::min(part, npx - part * t);
                for (size_t k = 0; k < n; ++k) {
                    out[4 * k] = src[3 * k];
                    out[4 * k + 1] = src[3 * k + 1];
                    out[4 * k + 2] = src[3 * k + 2];
                    out[4 * k + 3] = 1.0;
                }
                if (tm && t == 0) t_copied[i] = host_ms();
                continue;
            }
            const size_t part = (len[i] / nt + 4095) & ~(size_t)4095;
            if (part * t >= len[i]) continue;
            const size_t o = off[i] + part * t;
            std::memcpy((uint8_t*)dst + o, c->h_stage + o, std::min(part, len[i] - part * t));
            if (tm && t == 0) t_copied[i] = host_ms();
        }
        return hipSuccess;
    };
    std::vector<hipError_t> err(nt, hipSuccess);
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back([&, t] { err[t] = work(t); });
    err[0] = work(0);
    for (auto& t : th) t.join();
    if (tm) {
        fprintf(stderr, "copy_staged: %d pieces, from the call's wait (ms): ready/copied", npiece);
        for (int i = 0; i < npiece; ++i) fprintf(stderr, " %.3f/%.3f", t_ready[i] - t0, t_copied[i] - t0);
        fprintf(stderr, "; joined %.3f; nodes: staging %d..%d, frame %d..%d, device %d, this cpu %d\n", host_ms() - t0,
                page_node(c->h_stage), page_node(c->h_stage + off[npiece - 1] + len[npiece - 1] - 1), page_node(dst),
                page_node((uint8_t*)dst + (off[npiece - 1] + len[npiece - 1]) / (rgb ? 24 : 1) * (rgb ? 32 : 1) - 1), device_node(c->device), sched_getcpu());
    }
    for (hipError_t e : err)
        if (e != hipSuccess) return fail(MFX_E_DEVICE, std::string("readback: ") + hipGetErrorString(e));
    return MFX_OK;
}

static int stage_events(mfx_ctx* c) {
    for (int i = 0; i < kStageChunks; ++i) {
        if (!c->stage_ev[i]) HIPCHECK(hipEventCreateWithFlags(&c->stage_ev[i], hipEventDisableTiming));
        if (!c->band_ev[i]) HIPCHECK(hipEventCreateWithFlags(&c->band_ev[i], hipEventDisableTiming));
    }
    return MFX_OK;
}

// stream-ordered after what `st` has enqueued, complete on return; a small readback (or with no
// staging memory) is a plain copy
static int host_readback(mfx_ctx* c, void* dst, const void* src, size_t bytes, hipStream_t st) {
    const size_t kLarge = 16u << 20;
    if (bytes < kLarge || !ensure_stage(c, bytes)) {
        HIPCHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
        return MFX_OK;
    }
    int npiece = kStageChunks;  // MFX_READBACK_PIECES: A/B knob
    if (const char* e = getenv("MFX_READBACK_PIECES")) npiece = std::max(1, std::min(kStageChunks, atoi(e)));
    int rc = stage_events(c);
    if (rc) return rc;
    const size_t piece = (bytes / npiece + 4095) & ~(size_t)4095;
    size_t off[kStageChunks], len[kStageChunks];
    int used = 0;
    for (int i = 0; i < npiece && piece * i < bytes; ++i, ++used) {
        off[i] = piece * i;
        len[i] = std::min(piece, bytes - off[i]);
        HIPCHECK(hipMemcpyAsync(c->h_stage + off[i], (const uint8_t*)src + off[i], len[i], hipMemcpyDeviceToHost, st));
        HIPCHECK(hipEventRecord(c->stage_ev[i], st));
    }
    return copy_staged(c, dst, off, len, used);
}

int mfx_accum_read_mean(mfx_ctx* c, double count, double* frame) {
    if (!c || !frame) return fail(MFX_E_INVALID, "null argument");
    if (!(count > 0.0)) return fail(MFX_E_INVALID, "mfx_accum_read_mean: count must be > 0");
    // a device list whose last trace (a render call's included) has not been merged: merge it first,
    // so the mean covers every device's rows; a merged accumulator is not merged twice
    if (!c->accum_merged && (!c->peers.empty() || !c->comms.empty())) {
        const int rc = mfx_accum_reduce(c);
        if (rc) return rc;
    }
    HIPCHECK(hipSetDevice(c->device));
    // texture[i,j] <- color / float n (Integrators.fs:171): divided by the count itself
    HIPCHECK(mfx_launch_mean(c->d_accum, c->npix, count, c->d_frame, c->stream));
    return host_readback(c, frame, c->d_frame, 4 * sizeof(double) * (size_t)c->npix, c->stream);
}

int mfx_sync(mfx_ctx* c) {
    if (!c) return fail(MFX_E_STATE, "null context");
    for (mfx_ctx* d : devs_of(c)) {
        HIPCHECK(hipSetDevice(d->device));
        HIPCHECK(hipStreamSynchronize(d->stream));
    }
    return MFX_OK;
}

int mfx_stream(mfx_ctx* c, void** stream) {
    if (!c || !stream) return fail(MFX_E_INVALID, "null argument");
    *stream = (void*)c->stream;
    return MFX_OK;
}

static void sum_counters(const unsigned long long* h, double out[16]) {
    for (int k = 0; k < 16; ++k) {
        double v = 0;
        for (int g = 0; g < WF_SHARDS; ++g) v += (double)h[WF_NCTR * g + k];
        out[k] += v;
    }
    for (int d = 1; d < WF_ITER_CTRS; ++d)  // k_extend's per-iteration extension-ray counters
        for (int g = 0; g < WF_SHARDS; ++g) out[1] += (double)h[WF_NCTR * g + WF_CTR_ITER + d];
}

// MFX_RAY_QUEUE: the share of a trace's paths still live after each iteration (its extension rays
// over its paths), from counters read back after the trace; wf_trace moves the paths to ray queues
// from the first iteration that leaves fewer than WF_QUEUE_LIVE of them (the later bounces are the
// sparse ones). The decision only moves data: images are the same either way.
#define WF_QUEUE_LIVE 0.35
static void note_live(mfx_ctx* c, const unsigned long long* h) {
    double paths = 0, it[WF_ITER_CTRS] = {0};
    for (int g = 0; g < WF_SHARDS; ++g) {
        paths += (double)h[WF_NCTR * g + 0];
        for (int d = 1; d < WF_ITER_CTRS; ++d) it[d] += (double)h[WF_NCTR * g + WF_CTR_ITER + d];
    }
    if (paths <= 0 || it[1] <= 0) return;  // no wavefront trace (megakernel), or no path went on
    int from = -1;
    for (int d = 0; d + 1 < WF_ITER_CTRS && d < c->host.max_depth; ++d)
        if (it[d + 1] / paths < WF_QUEUE_LIVE) {
            from = d;
            break;
        }
    c->wf_queue_auto = from;
}

int mfx_ray_counts_total(mfx_ctx* c, double out[16], int32_t reset) {
    if (!c || !out) return fail(MFX_E_INVALID, "null argument");
    for (int k = 0; k < 16; ++k) out[k] = 0.0;
    for (mfx_ctx* d : devs_of(c)) {  // summed over the context's devices
        HIPCHECK(hipSetDevice(d->device));
        unsigned long long h[WF_NCTR * WF_SHARDS];
        HIPCHECK(hipMemcpyAsync(h, d->d_counters_total, sizeof(h), hipMemcpyDeviceToHost, d->stream));
        HIPCHECK(hipStreamSynchronize(d->stream));
        sum_counters(h, out);
        if (reset) HIPCHECK(hipMemsetAsync(d->d_counters_total, 0, sizeof(h), d->stream));
    }
    HIPCHECK(hipSetDevice(c->device));
    out[3] = out[0];  // paths == primary rays
    return MFX_OK;
}

int mfx_ray_counts(mfx_ctx* c, double out[16]) {
    if (!c || !out) return fail(MFX_E_INVALID, "null argument");
    if (c->rep_valid) {  // a call served from held frames (render-ahead)
        for (int k = 0; k < 16; ++k) out[k] = c->rep_counts[k];
        return MFX_OK;
    }
    for (int k = 0; k < 16; ++k) out[k] = 0.0;
    for (mfx_ctx* d : devs_of(c)) {  // summed over the context's devices
        HIPCHECK(hipSetDevice(d->device));
        unsigned long long h[WF_NCTR * WF_SHARDS];  // per-shard counter sets (the megakernel uses set 0)
        HIPCHECK(hipMemcpyAsync(h, d->d_counters, sizeof(h), hipMemcpyDeviceToHost, d->stream));
        HIPCHECK(hipStreamSynchronize(d->stream));
        sum_counters(h, out);
        note_live(d, h);
    }
    out[3] = out[0];  // paths == primary rays
    return MFX_OK;
}

// ---- render-ahead --------------------------------------------------------------------------------
// mfx_options.render_ahead = K > 1 with the whole sample set (part_count 1). Scene.Render
// (Scene.fs:331-333) asks for one sample per call: alone, a 1080p sample is ~21 rays per lane of a
// persistent grid plus the film/post launch and the readback per call. A sample's 1-spp image
// depends only on (seed, global sample index), so a call whose sample is not held traces the next K
// samples in one batched wavefront pass whose k_resolve runs, per pixel and in call order, each
// call's film add and post (the FP64 operations film_post_kernel runs per call, in the same order:
// k_resolve's frames mode) into K RGBA8 frames and the film after the last call: each call of the
// batch only copies its frame to the host. While a batch is served, the next one is traced in the
// background into the second buffer (the frame copies run on their own stream, so they overlap that
// trace). Every frame and the film are the bytes the one-sample path gives
// (tests/test_gpu_render_ahead.py). A buffer holds K frames (4 B per pixel each) and two films: no
// per-sample FP64 image is kept (round 3 kept one, 24 B per pixel per sample).
// Device lists: every device runs the same batches over its own band of tile rows, in its own
// buffers, film and copy stream, and a call copies each device's band rows of its frame straight
// into the caller's buffer: no FP64 buffer crosses devices, and the frames are the one-device bytes.
// The batch bookkeeping (base, n, expect, epoch, count0, reported) lives in the primary's ab[]; the
// peers' ab[] hold their device buffers only.
// The frames assume the calls follow each other with nothing else touching the film. A reset, a
// render call of spp != 1 or an mfx_sample call (which moves the sample sequence) bumps film_epoch
// after bringing d_film up to date; a held batch whose frames belong to an older epoch is traced
// again from the sample the next call needs. d_film is brought up to date by tracing, film only,
// the served samples it lacks (ahead_materialize): from the prefix of the batch it already holds
// (dfilm_n), else from the film before the batch — after a batch's last call it is a copy of the
// film after it. So a caller that alternates Render and mfx_film_mean re-traces each sample once.
static void ahead_free_all(mfx_ctx* c) {
    for (mfx_ctx* d : devs_of(c)) {
        (void)hipSetDevice(d->device);
        ahead_free(d);
    }
    (void)hipSetDevice(c->device);
    c->dfilm_buf = -1;
}

static int ahead_alloc(mfx_ctx* c) {
    const size_t plane = 3 * sizeof(double) * (size_t)c->npix, frame = 4 * (size_t)c->npix;
    const size_t per_sample = frame, fixed = 2 * plane + WF_NCTR * WF_SHARDS * sizeof(unsigned long long);
    // Both buffers within MFX_RENDER_AHEAD_MAX_BYTES (default 2 GiB) and a quarter of the free HBM
    // per device (shared by the contexts a device list puts on one GPU): a context never takes more
    // than that for render-ahead, whatever K it asked for. K shrinks to fit two buffers (the
    // background batch) while at least 8 samples fit in each; below that one buffer of as many
    // samples as fit. At 1080p (8.3 MB per sample, 100 MB of films per buffer) K = 64 takes 1.26 GB
    // for both. Every device of a list gets the same K (the tightest device's).
    size_t cap = (size_t)2 << 30;
    if (const char* e = getenv("MFX_RENDER_AHEAD_MAX_BYTES")) cap = std::min(cap, (size_t)atoll(e));
    const std::vector<mfx_ctx*> ds = devs_of(c);
    size_t budget = cap;
    for (mfx_ctx* d : ds) {
        size_t fr = 0, tot = 0;
        HIPCHECK(hipSetDevice(d->device));
        HIPCHECK(hipMemGetInfo(&fr, &tot));
        size_t share = 0;  // contexts of this list on the same GPU
        for (mfx_ctx* o : ds) share += o->device == d->device ? 1 : 0;
        budget = std::min(budget, std::min(fr / 4, cap) / share);
    }
    HIPCHECK(hipSetDevice(c->device));
    int nbuf = 2;
    int64_t k = std::min<int64_t>(c->render_ahead, budget / 2 > fixed ? (int64_t)((budget / 2 - fixed) / per_sample) : 0);
    if (k < std::min(8, c->render_ahead)) {
        nbuf = 1;  // no background batch: one buffer of as many samples as fit
        k = budget > fixed ? (int64_t)((budget - fixed) / per_sample) : 0;
        k = std::min<int64_t>(k, c->render_ahead);
    }
    if (k < 2) return MFX_E_NOMEM;
    hipError_t e = hipSuccess;
    for (mfx_ctx* d : ds) {
        e = hipSetDevice(d->device);
        for (int b = 0; b < nbuf && e == hipSuccess; ++b) {
            AheadBuf& B = d->ab[b];
            e = hipMalloc((void**)&B.frames, (size_t)k * frame);
            if (e == hipSuccess) e = hipMalloc((void**)&B.film_in, plane);
            if (e == hipSuccess) e = hipMalloc((void**)&B.film_out, plane);
            if (e == hipSuccess) e = hipMalloc((void**)&B.counters, WF_NCTR * WF_SHARDS * sizeof(unsigned long long));
            if (e == hipSuccess) e = hipEventCreate(&B.t0);
            if (e == hipSuccess) e = hipEventCreate(&B.t1);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&B.ready, hipEventDisableTiming);
        }
        if (e == hipSuccess) e = hipMalloc((void**)&d->d_counters_aux, WF_NCTR * WF_SHARDS * sizeof(unsigned long long));
        if (e == hipSuccess) e = hipEventCreate(&d->aux_ev0);
        if (e == hipSuccess) e = hipEventCreate(&d->aux_ev1);
        if (e != hipSuccess) break;
    }
    if (e != hipSuccess) {
        (void)hipGetLastError();
        ahead_free_all(c);
        return e == hipErrorOutOfMemory ? MFX_E_NOMEM : fail(MFX_E_DEVICE, std::string("render-ahead: ") + hipGetErrorString(e));
    }
    HIPCHECK(hipSetDevice(c->device));
    c->ab_nbuf = nbuf;
    c->ab_cap = (int)k;
    return MFX_OK;
}

// d_film (every device's) = the film as of the last render call: a copy of the film after the
// buffer's last call, or the film before the buffer (or the prefix of the buffer's samples it
// already holds) with the buffer's samples up to that call traced again, film only (the same
// paths, added in the same order: the same bits). Its rays are not reported (no call asked for them).
static int ahead_materialize(mfx_ctx* c) {
    if (c->film_in_dfilm) return MFX_OK;
    const int b = c->ab_cur;
    const AheadBuf& B = c->ab[b];
    const size_t plane = 3 * sizeof(double) * (size_t)c->npix;
    const int64_t want = c->ab_last_k + 1;  // the batch's samples the film holds
    const bool prefix = c->dfilm_buf == b && c->dfilm_n <= want;
    const int64_t from = want == B.n ? want : (prefix ? c->dfilm_n : 0);
    for (mfx_ctx* d : devs_of(c)) {
        HIPCHECK(hipSetDevice(d->device));
        const AheadBuf& D = d->ab[b];
        if (want == B.n) {
            HIPCHECK(hipMemcpyAsync(d->d_film, D.film_out, plane, hipMemcpyDeviceToDevice, d->stream));
            continue;
        }
        if (!prefix) HIPCHECK(hipMemcpyAsync(d->d_film, D.film_in, plane, hipMemcpyDeviceToDevice, d->stream));
        if (from == want || band_rows(d) == 0) continue;
        HIPCHECK(hipMemsetAsync(d->d_counters_aux, 0, WF_NCTR * WF_SHARDS * sizeof(unsigned long long), d->stream));
        const FrameMode fm{d->d_film, nullptr, 0.0};
        const int rc = wf_trace(d, want - from, B.base + from, &fm, d->d_counters_aux, d->aux_ev0, d->aux_ev1);
        if (rc) return rc;
    }
    HIPCHECK(hipSetDevice(c->device));
    c->dfilm_buf = b;
    c->dfilm_n = want;
    c->film_in_dfilm = true;
    return MFX_OK;
}

// the film leaves the held frames' sequence (a reset, an spp != 1 render call, mfx_sample)
static int ahead_break(mfx_ctx* c) {
    if (c->ab_nbuf == 0) return MFX_OK;
    const int rc = ahead_materialize(c);
    if (rc) return rc;
    c->film_epoch += 1;
    c->ab_cur = -1;
    return MFX_OK;
}

// trace samples [base, base + ab_cap) into buffer xi of every device: their frames from the film
// in buffer src's film_out (src < 0: d_film) with count0 = frameCount before them, and the film
// after them (enqueued only)
static int ahead_launch(mfx_ctx* c, int xi, int64_t base, int src, double count0) {
    const size_t plane = 3 * sizeof(double) * (size_t)c->npix;
    AheadBuf& B = c->ab[xi];
    B.base = base;
    B.n = c->ab_cap;
    B.reported = false;
    if (c->dfilm_buf == xi) c->dfilm_buf = -1;  // its film_in changes
    for (mfx_ctx* d : devs_of(c)) {
        HIPCHECK(hipSetDevice(d->device));
        AheadBuf& D = d->ab[xi];
        const double* film_src = src < 0 ? d->d_film : d->ab[src].film_out;
        HIPCHECK(hipMemcpyAsync(D.film_in, film_src, plane, hipMemcpyDeviceToDevice, d->stream));
        HIPCHECK(hipMemcpyAsync(D.film_out, film_src, plane, hipMemcpyDeviceToDevice, d->stream));
        HIPCHECK(hipMemsetAsync(D.counters, 0, WF_NCTR * WF_SHARDS * sizeof(unsigned long long), d->stream));
        if (band_rows(d) > 0) {
            const FrameMode fm{D.film_out, D.frames, count0};
            const int rc = wf_trace(d, B.n, base, &fm, D.counters, D.t0, D.t1);
            if (rc) {
                B.n = 0;
                (void)hipSetDevice(c->device);
                return rc;
            }
        } else {  // a device with no tile row: no rays in no time
            HIPCHECK(hipEventRecord(D.t0, d->stream));
            HIPCHECK(hipEventRecord(D.t1, d->stream));
        }
        HIPCHECK(hipEventRecord(D.ready, d->stream));
    }
    HIPCHECK(hipSetDevice(c->device));
    B.expect = 0;
    B.epoch = c->film_epoch;
    B.count0 = count0;
    if (src < 0) {  // film_in is d_film as it is
        c->dfilm_buf = xi;
        c->dfilm_n = 0;
    }
    return MFX_OK;
}

// A device's band rows of a y-major RGBA8 frame (device memory) into the caller's frame (host):
// one copy of the whole frame for a one-device context; on a device list two strided copies of its
// whole tile rows (band_tile_row: the even groups' rows and the odd groups' rows, each 8 rows every
// 2 * band_count * 8) plus the film's partial last tile row if it owns it.
static int copy_band_rgba(const mfx_ctx* d, uint8_t* dst, const uint8_t* src, hipStream_t st) {
    const int W = d->host.width, H = d->host.height;
    const size_t row = 4 * (size_t)W;
    if (d->band_count == 1) {
        HIPCHECK(hipMemcpyAsync(dst, src, row * (size_t)H, hipMemcpyDeviceToHost, st));
        return MFX_OK;
    }
    const int full = H / 8, tr = (H + 7) / 8, bi = d->band_index, bc = d->band_count;
    const int nb = band_row_count(bi, bc, tr);
    for (int k0 = 0; k0 < 2; ++k0) {
        int n = 0;  // the band's rows of this parity that are whole tile rows (a prefix: rows grow with k)
        for (int k = k0; k < nb && band_tile_row(bi, bc, k) < full; k += 2) ++n;
        if (n == 0) continue;
        const size_t off = (size_t)8 * band_tile_row(bi, bc, k0) * row, pitch = (size_t)16 * bc * row;
        HIPCHECK(hipMemcpy2DAsync(dst + off, pitch, src + off, pitch, 8 * row, (size_t)n, hipMemcpyDeviceToHost, st));
    }
    if (full < tr && nb > 0 && band_tile_row(bi, bc, nb - 1) == tr - 1) {
        const size_t off = (size_t)8 * full * row;
        HIPCHECK(hipMemcpyAsync(dst + off, src + off, (size_t)(H - 8 * full) * row, hipMemcpyDeviceToHost, st));
    }
    return MFX_OK;
}

// One render call (spp = 1) served from held frames. Returns MFX_E_NOMEM when no buffer fits (the
// caller then renders one sample per call, without render-ahead).
static int ahead_render(mfx_ctx* c, uint8_t* rgba) {
    if (c->ab_nbuf == 0) {
        const int rc = ahead_alloc(c);
        if (rc) return rc;
    }
    const int64_t s = c->next_sample;
    int xi = -1;
    for (int b = 0; b < c->ab_nbuf; ++b)
        if (c->ab[b].n > 0 && s >= c->ab[b].base && s < c->ab[b].base + c->ab[b].n) xi = b;
    int rc = MFX_OK;
    if (xi < 0) {  // not held: trace a batch from this sample, its frames from the film as it is
        rc = ahead_materialize(c);
        if (rc) return rc;
        xi = (c->ab_cur >= 0 && c->ab_nbuf == 2) ? 1 - c->ab_cur : 0;
        rc = ahead_launch(c, xi, s, -1, c->frame_count);
    } else if (c->ab[xi].epoch != c->film_epoch || c->ab[xi].expect != s - c->ab[xi].base) {
        rc = ahead_materialize(c);  // held, but the frames assumed another film: a batch from here
        if (!rc) rc = ahead_launch(c, xi, s, -1, c->frame_count);
    }
    if (rc) return rc;
    AheadBuf& X = c->ab[xi];
    const int64_t k = s - X.base;
    const std::vector<mfx_ctx*> ds = devs_of(c);
    // This call's frame, on each device's copy stream behind this batch's frames only: it overlaps
    // the background batch. Everything the call reads back goes there before the next batch is
    // enqueued, and the counters go to page-locked memory: a pageable copy enqueued behind the
    // background batch waited for it (r03b: 6,794 Mrays/s, 73 % of batch; r03c: 8,579, 93 %).
    const size_t frame = 4 * (size_t)c->npix;
    for (mfx_ctx* d : ds) {
        HIPCHECK(hipSetDevice(d->device));
        if (!d->copy_stream) HIPCHECK(hipStreamCreateWithFlags(&d->copy_stream, hipStreamNonBlocking));
        HIPCHECK(hipStreamWaitEvent(d->copy_stream, d->ab[xi].ready, 0));
        if (rgba) {
            const int rb = copy_band_rgba(d, rgba, d->ab[xi].frames + k * frame, d->copy_stream);
            if (rb) return rb;
        }
    }
    for (int q = 0; q < 16; ++q) c->rep_counts[q] = 0.0;
    c->rep_ms = 0.0;
    if (!X.reported) {  // the first call served from a batch reports its rays (all devices) and device time (the slowest)
        for (mfx_ctx* d : ds) {
            HIPCHECK(hipSetDevice(d->device));
            HIPCHECK(hipMemcpyAsync(d->h_counters, d->ab[xi].counters, WF_NCTR * WF_SHARDS * sizeof(unsigned long long),
                                    hipMemcpyDeviceToHost, d->copy_stream));
        }
        float worst = 0.f;
        for (mfx_ctx* d : ds) {
            HIPCHECK(hipSetDevice(d->device));
            HIPCHECK(hipStreamSynchronize(d->copy_stream));
            sum_counters(d->h_counters, c->rep_counts);
            note_live(d, d->h_counters);
            float f = 0.f;
            HIPCHECK(hipEventElapsedTime(&f, d->ab[xi].t0, d->ab[xi].t1));
            worst = std::max(worst, f);
        }
        c->rep_counts[3] = c->rep_counts[0];
        c->rep_ms = worst;
        X.reported = true;
    }
    for (mfx_ctx* d : ds) {
        HIPCHECK(hipSetDevice(d->device));
        HIPCHECK(hipStreamSynchronize(d->copy_stream));
    }
    HIPCHECK(hipSetDevice(c->device));
    c->rep_valid = true;
    c->ab_cur = xi;
    c->ab_last_k = k;
    X.expect = k + 1;
    c->film_in_dfilm = false;
    c->frame_count += 1.0;  // Film.AddSample: frameCount <- frameCount + 1 (Film.fs:19)
    c->next_sample += 1;
    if (c->ab_nbuf == 2) {  // the next batch, in the background, unless the other buffer holds it
        AheadBuf& Y = c->ab[1 - xi];
        const double count_end = X.count0 + (double)X.n;  // frameCount after X's last call
        // not held, or held but its frames assumed another film: traced (again) from X's film
        if (!(Y.n > 0 && Y.base == X.base + X.n) || Y.epoch != c->film_epoch || Y.count0 != count_end)
            rc = ahead_launch(c, 1 - xi, X.base + X.n, xi, count_end);
        // This call is served: a background batch that does not fit is not its failure (a NOMEM
        // here would make the caller render the call a second time). Y stays empty; the call
        // that needs it launches it, and falls back to one sample per call if it still fails.
        if (rc == MFX_E_NOMEM) {
            Y.n = 0;
            rc = MFX_OK;
        }
        if (rc) return rc;
    }
    return MFX_OK;
}

// mfx_sample on one device: the trace with its last resolve in column bands of tiles (ResolveSplit),
// each band's mean enqueued right behind its resolve and its readback on the copy stream, so the
// frame's DMA and the host copy overlap the rest of the resolve. A band of tile columns is a contiguous
// range of the x-major frame (pixel = x * h + y). The bits are the unbanded path's: a pixel's sum is
// its own thread's, and the mean is the same division. MFX_SAMPLE_BANDS=0: the unbanded path.
// Returns 1 (nothing done) when the call is not for it (a device list, no staging memory).
// mfx_sample's copy stream. MFX_COPY_PROBE=K (K > 1; an A/B knob, off by default) chooses it by
// measurement: K candidate streams each copy `bytes` (up to 16 MB) of the frame twice, the second copy
// timed, and the fastest is kept, once per context. The readback had run at ~53 GB/s in some contexts
// and ~26-31 GB/s in others; the probe found every candidate of a box alike (29.7 GB/s on one box,
// r06t: the rate is the box's, not the stream's), and contexts that probed traced 8 % slower in two
// cases of six (the streams it creates and destroys move the context's hardware queues; r06y, r06z),
// never without it. One stream, created at the first Sample call, is the default.
static int pick_copy_stream(mfx_ctx* c, size_t bytes) {
    int n = 1;
    if (const char* e = getenv("MFX_COPY_PROBE")) n = std::max(1, std::min(8, atoi(e)));
    if (n == 1) {
        HIPCHECK(hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
        return MFX_OK;
    }
    const size_t pb = std::min(bytes, (size_t)16 << 20);
    std::vector<hipStream_t> cand(n, nullptr);
    std::vector<float> ms(n, 1e30f);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    HIPCHECK(hipEventCreate(&e0));
    HIPCHECK(hipEventCreate(&e1));
    for (int i = 0; i < n; ++i) {
        HIPCHECK(hipStreamCreateWithFlags(&cand[i], hipStreamNonBlocking));
        HIPCHECK(hipMemcpyAsync(c->h_stage, c->d_frame, pb, hipMemcpyDeviceToHost, cand[i]));
        HIPCHECK(hipEventRecord(e0, cand[i]));
        HIPCHECK(hipMemcpyAsync(c->h_stage, c->d_frame, pb, hipMemcpyDeviceToHost, cand[i]));
        HIPCHECK(hipEventRecord(e1, cand[i]));
        HIPCHECK(hipEventSynchronize(e1));
        HIPCHECK(hipEventElapsedTime(&ms[i], e0, e1));
    }
    const int best = (int)(std::min_element(ms.begin(), ms.end()) - ms.begin());
    if (sample_timing()) {  // (diagnostics: the candidates' copies at once, k = 2 and all n)
        for (int k : {2, n}) {
            HIPCHECK(hipDeviceSynchronize());
            const double t0 = host_ms();
            for (int i = 0; i < k; ++i)
                HIPCHECK(hipMemcpyAsync(c->h_stage + (size_t)i * (pb / n), (const uint8_t*)c->d_frame, pb / n * (n / k),
                                        hipMemcpyDeviceToHost, cand[i]));
            for (int i = 0; i < k; ++i) HIPCHECK(hipStreamSynchronize(cand[i]));
            const double dt = host_ms() - t0;
            fprintf(stderr, "pick_copy_stream: %d streams at once, %zu B each: %.1f GB/s together\n", k, pb / n * (n / k),
                    (double)(pb / n * (n / k)) * k / (dt * 1e6));
        }
    }
    c->copy_stream = cand[best];
    for (int i = 0; i < n; ++i)
        if (i != best) HIPCHECK(hipStreamDestroy(cand[i]));
    HIPCHECK(hipEventDestroy(e0));
    HIPCHECK(hipEventDestroy(e1));
    if (sample_timing()) {
        fprintf(stderr, "pick_copy_stream: %zu B per probe, GB/s:", pb);
        for (int i = 0; i < n; ++i) fprintf(stderr, " %.1f", pb / (ms[i] * 1e6));
        fprintf(stderr, "; kept %d\n", best);
    }
    return MFX_OK;
}

static int sample_banded(mfx_ctx* c, int32_t spp, double* frame) {
    // 4 bands, one copy stream: in the bench process's state (r06i, scripts/sample_in_bench_probe.py)
    // 4 x 1 took 32.8-33.0 ms per C2 call, 8 x 1 33.0-33.2, 8 bands over two copy streams 33.7-33.9 and
    // the unbanded path 33.7 (a lone process: 8 x 1 32.1, unbanded 32.7, r06b)
    int nb = 4;
    if (const char* e = getenv("MFX_SAMPLE_BANDS")) nb = std::min(kStageChunks, atoi(e));
    const int W = c->host.width, H = c->host.height;
    nb = std::min(nb, (W + 7) / 8);
    // the means staged as interleaved RGB (MFX_SAMPLE_RGBA=1: the whole RGBA frame, A/B knob): the
    // host writes alpha while it copies, so the DMA carries 49.8 MB of C2's 66 MB frame
    const bool rgb = !(getenv("MFX_SAMPLE_RGBA") && atoi(getenv("MFX_SAMPLE_RGBA")) != 0);
    const size_t pxb = (rgb ? 3 : 4) * sizeof(double);
    const size_t bytes = pxb * (size_t)c->npix;
    if (nb < 1 || !c->peers.empty() || !c->comms.empty() || !ensure_stage(c, bytes)) return 1;
    HIPCHECK(hipSetDevice(c->device));
    int rc = stage_events(c);
    if (rc) return rc;
    if (!c->copy_stream) {
        rc = pick_copy_stream(c, bytes);
        if (rc) return rc;
    }
    int ncs = 1;  // MFX_SAMPLE_COPY_STREAMS=2: bands alternate over two copy streams (A/B knob; slower, r06i)
    if (const char* e = getenv("MFX_SAMPLE_COPY_STREAMS")) ncs = atoi(e) == 2 ? 2 : 1;
    // MFX_SAMPLE_ZEROCOPY=1 (A/B knob): each band's mean kernel runs on a copy stream and writes the
    // frame straight into the page-locked staging buffer across the fabric (no DMA)
    const bool zc = getenv("MFX_SAMPLE_ZEROCOPY") && atoi(getenv("MFX_SAMPLE_ZEROCOPY")) != 0;
    void* stage_dev = nullptr;  // the staging buffer's device address (zero-copy)
    if (zc) HIPCHECK(hipHostGetDevicePointer(&stage_dev, c->h_stage, 0));
    if (ncs == 2 && !c->sample_copy2) HIPCHECK(hipStreamCreateWithFlags(&c->sample_copy2, hipStreamNonBlocking));
    size_t off[kStageChunks] = {0}, len[kStageChunks] = {0};
    ResolveSplit S;
    S.nbands = nb;
    S.after = [&](int k, int tx0, int ntx) -> int {
        const int64_t p0 = (int64_t)tx0 * 8 * H, p1 = (int64_t)std::min(W, (tx0 + ntx) * 8) * H;
        off[k] = (size_t)p0 * pxb;
        len[k] = (size_t)(p1 - p0) * pxb;
        hipStream_t cs = (ncs == 2 && (k & 1)) ? c->sample_copy2 : c->copy_stream;
        auto mean = [&](double* out, hipStream_t st) {
            return rgb ? mfx_launch_mean_rgb(c->d_accum, c->npix, (double)spp, out, st, p0, p1)
                       : mfx_launch_mean(c->d_accum, c->npix, (double)spp, out, st, p0, p1);
        };
        if (zc) {
            HIPCHECK(hipEventRecord(c->band_ev[k], c->stream));
            HIPCHECK(hipStreamWaitEvent(cs, c->band_ev[k], 0));
            HIPCHECK(mean((double*)stage_dev, cs));
        } else {
            HIPCHECK(mean(c->d_frame, c->stream));
            HIPCHECK(hipEventRecord(c->band_ev[k], c->stream));
            HIPCHECK(hipStreamWaitEvent(cs, c->band_ev[k], 0));
            if (len[k]) HIPCHECK(hipMemcpyAsync(c->h_stage + off[k], (const uint8_t*)c->d_frame + off[k], len[k],
                                                hipMemcpyDeviceToHost, cs));
        }
        HIPCHECK(hipEventRecord(c->stage_ev[k], cs));
        return MFX_OK;
    };
    c->rep_valid = false;
    c->accum_merged = false;
    const double t0 = sample_timing() ? host_ms() : 0.0;
    rc = dev_trace_accumulate(c, spp, c->next_sample, &S);
    if (rc) return rc;
    rc = settle_queue_auto(c);
    if (rc) return rc;
    c->next_sample += spp;
    if (!S.used) {  // (one sample per pixel: the megakernel ran, no banded resolve)
        rc = mfx_accum_read_mean(c, (double)spp, frame);
        return rc ? rc : mfx_sync(c);
    }
    if (sample_timing()) fprintf(stderr, "sample_banded: enqueued in %.3f ms\n", host_ms() - t0);
    rc = copy_staged(c, frame, off, len, nb, rgb);
    if (rc) return rc;
    rc = mfx_sync(c);
    if (sample_timing()) fprintf(stderr, "sample_banded: call %.3f ms\n", host_ms() - t0);
    return rc;
}

int mfx_sample(mfx_ctx* c, int32_t spp, double* frame) {
    if (!c || !frame) return fail(MFX_E_INVALID, "null argument");
    if (c->api_part_count != 1)
        return fail(MFX_E_STATE, "mfx_sample needs the whole film and sample set (part_count == 1); "
                                 "partitioned contexts compose with mfx_trace_accumulate + a reduce");
    if (spp < 1) return fail(MFX_E_INVALID, "spp must be >= 1");
    int rc = ahead_break(c);  // it moves the sample sequence past held frames
    if (rc) return rc;
    rc = mfx_accum_clear(c);
    if (rc) return rc;
    rc = sample_banded(c, spp, frame);
    if (rc != 1) return rc;
    rc = mfx_trace_accumulate(c, spp, c->next_sample);
    if (rc) return rc;
    c->next_sample += spp;
    rc = mfx_accum_reduce(c);  // a device list: its bands merged into the primary's accumulator
    if (rc) return rc;
    rc = mfx_accum_read_mean(c, (double)spp, frame);
    if (rc) return rc;
    return mfx_sync(c);
}

// Without render-ahead (or spp != 1): every device traces its band into its accumulator, adds it
// to its band of the film and post-processes it (film_post_kernel), and copies its band rows of
// the RGBA8 frame to the caller's buffer. No device buffer is reduced: each pixel's film lives on
// the device whose band holds it (mfx_film_mean merges them).
int mfx_render_rgba8(mfx_ctx* c, int32_t spp, uint8_t* rgba) {
    if (!c) return fail(MFX_E_INVALID, "null context");
    if (c->api_part_count != 1) return fail(MFX_E_STATE, "mfx_render_rgba8 needs part_count == 1");
    if (spp < 1) return fail(MFX_E_INVALID, "spp must be >= 1");
    if (spp == 1 && c->render_ahead > 1) {
        HIPCHECK(hipSetDevice(c->device));
        const int rc = ahead_render(c, rgba);
        if (rc != MFX_E_NOMEM) return rc;
        // no room for the batch (nothing of this call was served): this context renders one
        // sample per call from now on; the film comes back to d_film and the buffers are freed
        c->render_ahead = 0;
        const int rb = ahead_break(c);
        if (rb) return rb;
        ahead_free_all(c);
    }
    int rc = ahead_break(c);
    if (rc) return rc;
    rc = mfx_accum_clear(c);
    if (rc) return rc;
    rc = mfx_trace_accumulate(c, spp, c->next_sample);
    if (rc) return rc;
    c->next_sample += spp;
    c->frame_count += 1.0;  // Film.AddSample: frameCount <- frameCount + 1 (Film.fs:19)
    c->dfilm_buf = -1;      // d_film moves on
    const std::vector<mfx_ctx*> ds = devs_of(c);
    for (mfx_ctx* d : ds) {
        HIPCHECK(hipSetDevice(d->device));
        HIPCHECK(mfx_launch_film_post(d->d_accum, d->d_film, c->host.width, c->host.height, (double)spp, c->frame_count, 1,
                                      rgba ? d->d_rgba : nullptr, d->stream));
        if (rgba) {
            const int rb = copy_band_rgba(d, rgba, d->d_rgba, d->stream);
            if (rb) return rb;
        }
    }
    return mfx_sync(c);
}

int mfx_accumulate_render_rgba8(mfx_ctx* c, int32_t spp, uint8_t* rgba) { return mfx_render_rgba8(c, spp, rgba); }

int mfx_stats(mfx_ctx* c, double* rays, double* seconds) {
    if (!c) return fail(MFX_E_INVALID, "null context");
    if (seconds) {
        double ms = 0;
        int rc = mfx_last_trace_ms(c, &ms);
        if (rc) return rc;
        *seconds = ms * 1e-3;
    }
    if (rays) {
        double n[16];
        int rc = mfx_ray_counts(c, n);
        if (rc) return rc;
        *rays = n[0] + n[1] + n[2];
    }
    return MFX_OK;
}

int mfx_reset(mfx_ctx* c) {
    if (!c) return fail(MFX_E_STATE, "null context");
    // stream-ordered after anything that reads the film (no wait for a background batch)
    for (mfx_ctx* d : devs_of(c)) {
        HIPCHECK(hipSetDevice(d->device));
        HIPCHECK(hipMemsetAsync(d->d_film, 0, 3 * sizeof(double) * (size_t)d->npix, d->stream));
    }
    HIPCHECK(hipSetDevice(c->device));
    c->frame_count = 0.0;
    c->film_in_dfilm = true;
    c->dfilm_buf = -1;
    if (c->ab_nbuf) {
        c->film_epoch += 1;
        c->ab_cur = -1;
        return MFX_OK;
    }
    return mfx_sync(c);
}

int mfx_film_mean(mfx_ctx* c, double* frame) {
    if (!c || !frame) return fail(MFX_E_INVALID, "null argument");
    HIPCHECK(hipSetDevice(c->device));
    int rc = ahead_materialize(c);
    if (rc) return rc;
    const double* film = c->d_film;
    if (!c->peers.empty() || !c->comms.empty()) {  // a device list: the devices' bands of the film, merged
        if (!c->d_merge) HIPCHECK(hipMalloc((void**)&c->d_merge, 3 * sizeof(double) * (size_t)c->npix));
        rc = reduce_planes(c, [](mfx_ctx* d) { return d->d_film; }, c->d_merge, "mfx_film_mean");
        if (rc) return rc;
        film = c->d_merge;
    }
    HIPCHECK(mfx_launch_film_mean(film, c->npix, c->frame_count, c->d_frame, c->stream));
    return host_readback(c, frame, c->d_frame, 4 * sizeof(double) * (size_t)c->npix, c->stream);
}

static int run_query(mfx_ctx* c, int64_t n, const double* rays, double tmin, double tmax, const double* tmax_arr,
                     double* t_out, int32_t* prim_out, double* normal_out, int32_t* occ_out, bool shadow) {
    if (!c || !rays || n < 0) return fail(MFX_E_INVALID, "bad query arguments");
    if (n == 0) return MFX_OK;
    HIPCHECK(hipSetDevice(c->device));
    double *d_rays = nullptr, *d_tmax = nullptr, *d_t = nullptr, *d_n = nullptr;
    int32_t *d_p = nullptr, *d_o = nullptr;
    hipError_t e = hipMalloc((void**)&d_rays, sizeof(double) * 6 * n);
    if (e == hipSuccess) e = hipMemcpy(d_rays, rays, sizeof(double) * 6 * n, hipMemcpyHostToDevice);
    if (e == hipSuccess && shadow) e = hipMalloc((void**)&d_tmax, sizeof(double) * n);
    if (e == hipSuccess && shadow) e = hipMemcpy(d_tmax, tmax_arr, sizeof(double) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess && shadow) e = hipMalloc((void**)&d_o, sizeof(int32_t) * n);
    if (e == hipSuccess && !shadow) e = hipMalloc((void**)&d_t, sizeof(double) * n);
    if (e == hipSuccess && !shadow) e = hipMalloc((void**)&d_p, sizeof(int32_t) * n);
    if (e == hipSuccess && !shadow) e = hipMalloc((void**)&d_n, sizeof(double) * 3 * n);
    if (e == hipSuccess) {
        QueryParams Q;
        std::memset(&Q, 0, sizeof(Q));
        Q.nodes = c->d_nodes;
        Q.slots = c->d_slots;
    Q.slot_ref = c->d_slot_ref;
        Q.ref_blob = c->d_ref_blob;
        Q.shade = c->d_shade;
        Q.inst = c->d_inst;
        Q.rays = d_rays;
        Q.tmax_per_ray = d_tmax;
        Q.t_out = d_t;
        Q.prim_out = d_p;
        Q.normal_out = d_n;
        Q.occ_out = d_o;
        Q.n = n;
        Q.tmin = tmin;
        Q.tmax = tmax;
        Q.stack_size = c->stack_size;
        e = mfx_launch_query(Q, shadow, c->stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess && shadow) e = hipMemcpy(occ_out, d_o, sizeof(int32_t) * n, hipMemcpyDeviceToHost);
    if (e == hipSuccess && !shadow) e = hipMemcpy(t_out, d_t, sizeof(double) * n, hipMemcpyDeviceToHost);
    if (e == hipSuccess && !shadow) e = hipMemcpy(prim_out, d_p, sizeof(int32_t) * n, hipMemcpyDeviceToHost);
    if (e == hipSuccess && !shadow && normal_out)
        e = hipMemcpy(normal_out, d_n, sizeof(double) * 3 * n, hipMemcpyDeviceToHost);
    for (void* b : {(void*)d_rays, (void*)d_tmax, (void*)d_t, (void*)d_n, (void*)d_p, (void*)d_o})
        if (b) (void)hipFree(b);
    if (e != hipSuccess) return fail(MFX_E_DEVICE, std::string("query: ") + hipGetErrorString(e));
    return MFX_OK;
}

int mfx_closest_hit(mfx_ctx* c, int64_t n, const double* rays, double tmin, double tmax, double* t_out,
                    int32_t* prim_out, double* normal_out) {
    if (!t_out || !prim_out) return fail(MFX_E_INVALID, "null output");
    return run_query(c, n, rays, tmin, tmax, nullptr, t_out, prim_out, normal_out, nullptr, false);
}

int mfx_any_hit(mfx_ctx* c, int64_t n, const double* rays, double tmin, const double* tmax, int32_t* occluded_out) {
    if (!tmax || !occluded_out) return fail(MFX_E_INVALID, "null argument");
    return run_query(c, n, rays, tmin, 0.0, tmax, nullptr, nullptr, nullptr, occluded_out, true);
}

int mfx_ref_leaves(mfx_ctx* c, int32_t* indices_out, int32_t* leaf_first_out, int32_t* leaf_count_out,
                   int32_t* nleaves_out) {
    if (!c || !indices_out || !leaf_first_out || !leaf_count_out || !nleaves_out)
        return fail(MFX_E_INVALID, "null argument");
    std::copy(c->host.ref_indices.begin(), c->host.ref_indices.end(), indices_out);
    std::copy(c->host.leaf_first.begin(), c->host.leaf_first.end(), leaf_first_out);
    std::copy(c->host.leaf_count.begin(), c->host.leaf_count.end(), leaf_count_out);
    *nleaves_out = (int32_t)c->host.leaf_first.size();
    return MFX_OK;
}

int mfx_build_info(mfx_ctx* c, double out[8], uint64_t* digest) {
    if (!c) return fail(MFX_E_STATE, "null context");
    const MfxHostScene& h = c->host;
    if (out) {
        out[0] = h.ms_ref_bvh;
        out[1] = h.ms_bvh;
        out[2] = h.ms_total;
        out[3] = h.images_gpu ? 2.0 : (h.bvh_gpu ? 1.0 : 0.0);
        out[4] = (double)h.nodes.size();
        out[5] = (double)h.slots.size();
        out[6] = h.nodes2;
        out[7] = h.bvh_levels;
    }
    if (digest) {  // FNV-1a over the device images
        uint64_t x = 1469598103934665603ULL;
        auto mix = [&](const void* p, size_t n) {
            const uint8_t* b = (const uint8_t*)p;
            for (size_t i = 0; i < n; ++i) x = (x ^ b[i]) * 1099511628211ULL;
        };
        mix(h.nodes.data(), h.nodes.size() * sizeof(MfxNode));
        mix(h.slots.data(), h.slots.size() * sizeof(MfxSlot));
        mix(h.slot_ref.data(), h.slot_ref.size() * sizeof(int32_t));
        mix(h.ref_blob.data(), h.ref_blob.size());
        mix(h.shade.data(), h.shade.size() * sizeof(MfxShade));
        mix(h.inst.data(), h.inst.size() * sizeof(MfxInstance));
        *digest = x;
    }
    return MFX_OK;
}

int mfx_device_info(mfx_ctx* c, int32_t* out, int32_t cap) {
    if (!c || !out) return fail(MFX_E_INVALID, "null argument");
    const std::vector<mfx_ctx*> ds = devs_of(c);
    if (cap < 5 + (int32_t)ds.size()) return fail(MFX_E_INVALID, "mfx_device_info: cap < 5 + devices");
    out[0] = (int32_t)ds.size();
    out[1] = (int32_t)c->comms.size();
    out[2] = !c->comms.empty() ? 1 : (c->peers.empty() ? 0 : 2);
    out[3] = c->band_index;
    out[4] = c->band_count;
    for (size_t g = 0; g < ds.size(); ++g) out[5 + g] = ds[g]->device;
    return MFX_OK;
}

int mfx_build_leaves(const mfx_scene_desc* scene, int32_t* indices_out, int32_t* leaf_first_out,
                     int32_t* leaf_count_out, int32_t* nleaves_out, int32_t info_out[4]) {
    MfxHostScene s;
    std::string err;
    if (!mfx_build_scene(scene, s, err)) return fail(MFX_E_INVALID, "mfx_build_leaves: " + err);
    if (indices_out) std::copy(s.ref_indices.begin(), s.ref_indices.end(), indices_out);
    if (leaf_first_out) std::copy(s.leaf_first.begin(), s.leaf_first.end(), leaf_first_out);
    if (leaf_count_out) std::copy(s.leaf_count.begin(), s.leaf_count.end(), leaf_count_out);
    if (nleaves_out) *nleaves_out = (int32_t)s.leaf_first.size();
    if (info_out) {
        info_out[0] = s.nclusters;
        info_out[1] = (int32_t)s.nodes.size();
        info_out[2] = s.stack_entries;
        info_out[3] = (int32_t)s.slots.size();
    }
    return MFX_OK;
}

int mfx_fp64_selftest(int32_t device, int64_t n, const double* a, const double* b, double* div_out, double* sqrt_out) {
    if (n <= 0 || !a || !b || !div_out || !sqrt_out) return fail(MFX_E_INVALID, "bad selftest arguments");
    HIPCHECK(hipSetDevice(device));
    double *da = nullptr, *db = nullptr, *dd = nullptr, *ds = nullptr;
    const size_t bytes = sizeof(double) * n;
    hipError_t e = hipMalloc((void**)&da, bytes);
    if (e == hipSuccess) e = hipMalloc((void**)&db, bytes);
    if (e == hipSuccess) e = hipMalloc((void**)&dd, bytes);
    if (e == hipSuccess) e = hipMalloc((void**)&ds, bytes);
    if (e == hipSuccess) e = hipMemcpy(da, a, bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(db, b, bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = mfx_launch_fp64_selftest(da, db, n, dd, ds, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(div_out, dd, bytes, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(sqrt_out, ds, bytes, hipMemcpyDeviceToHost);
    for (void* p : {(void*)da, (void*)db, (void*)dd, (void*)ds})
        if (p) (void)hipFree(p);
    if (e != hipSuccess) return fail(MFX_E_DEVICE, std::string("fp64 selftest: ") + hipGetErrorString(e));
    return MFX_OK;
}

int mfx_aabb_selftest(int32_t device, int64_t n, const double* rec, int32_t* out) {
    if (n <= 0 || !rec || !out) return fail(MFX_E_INVALID, "bad selftest arguments");
    HIPCHECK(hipSetDevice(device));
    double* dr = nullptr;
    int32_t* dout = nullptr;
    hipError_t e = hipMalloc((void**)&dr, sizeof(double) * 24 * n);
    if (e == hipSuccess) e = hipMalloc((void**)&dout, sizeof(int32_t) * 3 * n);
    if (e == hipSuccess) e = hipMemcpy(dr, rec, sizeof(double) * 24 * n, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = mfx_launch_aabb_selftest(dr, n, dout, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(out, dout, sizeof(int32_t) * 3 * n, hipMemcpyDeviceToHost);
    if (dr) (void)hipFree(dr);
    if (dout) (void)hipFree(dout);
    if (e != hipSuccess) return fail(MFX_E_DEVICE, std::string("aabb selftest: ") + hipGetErrorString(e));
    return MFX_OK;
}

}  // extern "C"
