// smem_gpu.cpp — runtime behind the C ABI in include/smem_gpu.h.
//
// Replaces the reference's accelerator plumbing:
//   * AAL runtime + 3 GB shared buffer + CSR writes (software/HelloALINLB.cpp:254-485)
//     -> one HIP device context per smem_gpu_t, index resident in HBM;
//   * the FPGA index upload (software/bwa.c:286-307) -> smem_gpu_init;
//   * the HARP manager thread that serialises every worker's batch through
//     one FPGA buffer with polled hand-shakes (software/fastmap.c:320-429)
//     -> per-worker smem_batch_t objects, each with its own HIP stream and
//     device buffers, so concurrent kt_for_batch workers never wait on a
//     manager and never get rejected.
#include <hip/hip_runtime.h>
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <string>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <future>
#include <mutex>
#include <new>
#include <thread>
#include <unordered_map>
#include <vector>

#include "smem_gpu.h"
#include "smem_kernels.h"
#include "chain_kernels.h"
#include "ksw_kernels.h"
#include "aln_kernels.h"

using smem::CallRec;
using smem::Intv;

static_assert(sizeof(Intv) == sizeof(smem_intv_t), "interval layout");

namespace {

thread_local char g_err[512];
// set when a HIP call of this thread's current entry point failed with a
// runtime error (not an allocation failure): the device is then marked
// faulted when the call leaves (see DeviceCall)
thread_local int g_hip_fault = 0;
// the library's own warm-up calls are not counted by SMEM_GPU_FAIL
thread_local int g_no_inject = 0;
// SMEM_GPU_TIMES diagnostics: this thread's seconds waiting for the device's
// upload chain (gpu_wait) and for an admitted stream pair
thread_local double g_t_ready = 0, g_t_admit = 0;
static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static const double g_t_lib = now_s();  // the library's load (for a linked binary: its start)
// SMEM_GPU_TIMES: time spent releasing batch buffers (device / pinned host) and their counts
static std::atomic<int64_t> g_rel_dev_ns{0}, g_rel_host_ns{0}, g_rel_dev_n{0}, g_rel_host_n{0};

// runtime errors after which the device (or its context) cannot be trusted:
// a kernel fault, a lost or uninitialised device, a context gone; every later
// call is refused.  Others -- a launch's configuration or an argument the
// runtime rejected (hipErrorInvalidValue, hipErrorInvalidConfiguration, ...)
// -- refuse that one call and leave the device usable.
bool hip_error_breaks_device(hipError_t e) {
    switch (e) {
        case hipErrorLaunchFailure: case hipErrorIllegalAddress: case hipErrorECCNotCorrectable:
        case hipErrorAssert: case hipErrorNoDevice: case hipErrorLaunchTimeOut: case hipErrorContextIsDestroyed:
        case hipErrorNotInitialized: case hipErrorDeinitialized: case hipErrorIllegalState: case hipErrorUnknown:
            return true;
        default:
            return false;
    }
}

int fail(int code, const char* what, hipError_t e = hipSuccess) {
    if (e != hipSuccess)
        snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
    else
        snprintf(g_err, sizeof(g_err), "%s", what);
    // an allocation that does not fit is a refusal, not a broken device
    if (code == SMEM_E_DEVICE && e == hipErrorOutOfMemory) return SMEM_E_NOMEM;
    if (code == SMEM_E_DEVICE && hip_error_breaks_device(e)) g_hip_fault = 1;
    return code;
}

// SMEM_GPU_FAIL=<stage>:<k>[:sticky|:hip=<code>] -- fault injection for the
// reject -> CPU path: every k-th call (process-wide) of the stage returns
// SMEM_E_DEVICE after its work is enqueued and before it is waited for, so
// the drain on the way out is what keeps that work from landing after the
// caller resumed.  stage: upload (smem_batch_set_reads*), seed
// (smem_batch_run), sa, chain, aln (smem_batch_chain2aln), fetch, or any.
// ":sticky" also marks the device faulted, as a real runtime failure does;
// ":hip=<code>" goes through fail() with that hipError_t, so the
// classification decides (hip=9, hipErrorInvalidConfiguration: that call only;
// hip=719, hipErrorLaunchFailure: the device).
enum { ST_UPLOAD, ST_SEED, ST_SA, ST_CHAIN, ST_ALN, ST_FETCH, ST_N };
const char* const k_stage_name[ST_N] = {"upload", "seed", "sa", "chain", "aln", "fetch"};
std::atomic<uint64_t> g_stage_calls[ST_N];

int inject_fault(int stage) {
    const char* e = getenv("SMEM_GPU_FAIL");
    if (!e || !*e || g_no_inject) return SMEM_OK;
    const char* c = strchr(e, ':');
    if (!c) return SMEM_OK;
    const std::string name(e, (size_t)(c - e));
    if (name != "any" && name != k_stage_name[stage]) return SMEM_OK;
    const long k = strtol(c + 1, nullptr, 10);
    if (k <= 0) return SMEM_OK;
    const uint64_t n = g_stage_calls[stage].fetch_add(1) + 1;
    if (n % (uint64_t)k) return SMEM_OK;
    snprintf(g_err, sizeof(g_err), "injected failure (SMEM_GPU_FAIL=%s): stage %s, call %llu", e, k_stage_name[stage],
             (unsigned long long)n);
    if (strstr(c + 1, ":sticky")) g_hip_fault = 2;
    if (const char* h = strstr(c + 1, ":hip=")) {
        char what[256];
        snprintf(what, sizeof(what), "%s", g_err);
        return fail(SMEM_E_DEVICE, what, (hipError_t)atoi(h + 5));
    }
    return SMEM_E_DEVICE;
}

#define INJECT(stage)                                   \
    do {                                                \
        if (int _r = inject_fault(stage)) return _r;    \
    } while (0)

#define HIP_TRY(expr)                                                   \
    do {                                                                \
        hipError_t _e = (expr);                                         \
        if (_e != hipSuccess) return fail(SMEM_E_DEVICE, #expr, _e);    \
    } while (0)

// A worker slot's buffers carved from two blocks (device, pinned host)
// instead of ~80 separate allocations: each hipFree / hipHostFree is a
// driver round trip (~1 ms and ~3 ms each, profiles/r04/e2e), so releasing 16
// slots one buffer at a time took 0.3 s of `bwa mem`'s exit.  Used by
// smem_gpu_reserve_slots (the sizes are known there: a measuring pass
// records them, then the blocks are allocated and the same calls carve);
// buffers that grow later get their own allocation, as without.
struct Arena {
    bool measure = false;
    char* base = nullptr;
    size_t cap = 0, used = 0;
    void* take(size_t bytes) {
        const size_t at = (used + 255) & ~(size_t)255;
        if (measure) {
            used = at + bytes;
            return reinterpret_cast<void*>((uintptr_t)256);  // never dereferenced, never freed
        }
        if (!base || at + bytes > cap) return nullptr;
        used = at + bytes;
        return base + at;
    }
};
thread_local Arena* t_dev_arena = nullptr;
thread_local Arena* t_host_arena = nullptr;

// SMEM_GPU_GUARD=1 (diagnostics): every device buffer allocated on its own is followed by
// GUARD_BYTES of a known pattern, checked after each call on a batch (guard_check): a kernel
// writing past the end of its buffer is named by the buffer's place in batch_bufs' order
constexpr size_t GUARD_BYTES = 64 << 10;
static bool guard_on() {
    static const bool on = getenv("SMEM_GPU_GUARD") && atoi(getenv("SMEM_GPU_GUARD"));
    return on;
}

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    bool own = true;  // false: carved from the slot's block
    hipError_t ensure(size_t want) {
        if (want <= n && p) return hipSuccess;
        release();
        const size_t m = std::max<size_t>(want, 1);
        if (t_dev_arena)
            if (void* a = t_dev_arena->take(m * sizeof(T))) {
                p = static_cast<T*>(a), n = m, own = false;
                return hipSuccess;
            }
        const size_t extra = guard_on() ? GUARD_BYTES : 0;
        hipError_t e = hipMalloc(&p, m * sizeof(T) + extra);
        if (e == hipSuccess && extra) e = hipMemset(reinterpret_cast<char*>(p) + m * sizeof(T), 0xA5, extra);
        if (e == hipSuccess) n = m, own = true;
        return e;
    }
    // ensure() with 25 % headroom when it must reallocate: for scratch whose
    // size follows each batch's contents (a reallocation frees, and hipFree
    // waits for the whole device)
    hipError_t grow(size_t want) {
        if (want <= n && p) return hipSuccess;
        return ensure(want + want / 4);
    }
    void release() {
        if (p && own) (void)hipFree(p);
        p = nullptr;
        n = 0;
        own = true;
    }
    uint64_t bytes() const { return p ? (uint64_t)n * sizeof(T) : 0; }
};

template <class T>
struct HostBuf {
    T* p = nullptr;
    size_t n = 0;
    bool own = true;
    // a pinned result buffer of at least `want` elements, grown with 25 %
    // headroom: batches of a worker vary in size, and re-pinning on every
    // slightly larger one costs more than the copy
    hipError_t grow(size_t want) {
        if (want <= n && p) return hipSuccess;
        return ensure(want + want / 4);
    }
    hipError_t ensure(size_t want) {
        if (want <= n && p) return hipSuccess;
        release();
        const size_t m = std::max<size_t>(want, 1);
        if (t_host_arena)
            if (void* a = t_host_arena->take(m * sizeof(T))) {
                p = static_cast<T*>(a), n = m, own = false;
                return hipSuccess;
            }
        hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&p), m * sizeof(T), hipHostMallocDefault);
        if (e == hipSuccess) n = m, own = true;
        return e;
    }
    void release() {
        if (p && own) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
        own = true;
    }
    uint64_t bytes() const { return p ? (uint64_t)n * sizeof(T) : 0; }
};

}  // namespace

extern "C" hipError_t smem_preload_seed(void);
extern "C" hipError_t smem_preload_chain(void);
extern "C" hipError_t smem_preload_ksw(void);
extern "C" hipError_t smem_preload_aln(void);

// device SA sampling interval = 2^SA_DENSE_SHIFT (see smem_gpu_load_sa)
constexpr uint32_t SA_DENSE_SHIFT = 2;
// chaining: reads with more seed occurrences than this get a wave each
// (chain_heavy_kernel), giants first; its chain tree / filter records live
// in CHAIN_HEAVY_LDS bytes of LDS (one such workgroup per CU)
constexpr uint32_t CHAIN_HEAVY_MIN = 16, CHAIN_GIANT_MIN = 2048, CHAIN_HEAVY_LDS = 150 * 1024,
                   CHAIN_REST_LDS = 28 * 1024;

// the seeding kernel a handle starts with: seed_wp_kernel<24 owners per wave, 18 LDS
// list entries, 4 blocks per CU> (variant 49; variant 2 is the
// lane-per-read seed_kernel of rounds 1-4)
constexpr int kSeedDefault = 49;
// the persistent grid's lanes per CU when the caller sets none: 4 blocks of 256
// fit the 4-block variants' LDS, but a grid of exactly 4 per CU leaves no VGPR
// room for the finalize / compaction kernels of another batch (measured: the
// steps then serialise), so 3.75 (profiles/r05/ab_wp)
static int seed_lanes_per_cu(int variant) {
    switch (variant) {
        case 44: case 45: case 46: case 49: case 50: case 51: case 52: case 53: case 54: case 56: case 57:
        case 58: case 59: case 60: case 61: case 62: return 960;
        default: return 768;
    }
}
// lanes a launch gives each read: seed_wp_kernel's waves own 32 (variant 42: 24) reads
// reads a wave of the seeding kernel owns at once (seed_wp_kernel<OWN, ...>; seed_kernel: one per lane)
static int seed_owners_per_wave(int variant) {
    switch (variant) {
        case 40: case 41: case 43: case 45: case 47: case 55: return 32;
        case 42: case 44: case 48: case 49: case 51: case 52: case 54: case 56: case 57:
        case 58: case 59: case 60: case 61: case 62: return 24;
        case 46: case 53: return 28;
        case 50: return 20;
        default: return 64;
    }
}
// lanes a launch gives each read so that every owner of a small batch's grid has one
static int seed_lanes_per_read(int variant) { return (64 + seed_owners_per_wave(variant) - 1) / seed_owners_per_wave(variant); }
// list arenas a launch of `lanes` lanes addresses (2 x cap_list packed entries each): seed_wp_kernel
// one per owner (OWN a wave), seed_kernel one per lane
static size_t seed_arenas(int variant, int lanes) {
#ifdef SMEM_WP_ARENA_PER_LANE
    (void)variant;
    return (size_t)lanes;
#else
    return variant >= 40 ? (size_t)(lanes / 64) * (size_t)seed_owners_per_wave(variant) : (size_t)lanes;
#endif
}

struct smem_gpu {
    int device = 0;
    int n_cu = 0;
    int lanes_per_cu = 0;  // 0: the seeding kernel's own (seed_lanes_per_cu)
    int intv_cap = 0;
    int variant = kSeedDefault;  // see smem_gpu_set_kernel_variant
    uint32_t* d_bwt = nullptr;      // reference layout (A/B variants 3, 4; freed after the Occ64 re-layout otherwise)
    uint32_t* d_occ64 = nullptr;    // Occ64 layout (default kernel)
    uint32_t* d_occ192 = nullptr;   // Occ192 layout (variant 10)
    uint4* d_kt = nullptr;          // k-mer bi-interval table (smem_gpu_set_kmer_table; variant 23)
    int kt_k = 0;
    uint64_t* d_sa = nullptr;       // sampled SA (smem_gpu_load_sa), n_sa + 1 words
    uint8_t* d_pac = nullptr;       // 2-bit forward strand (smem_gpu_load_pac)
    int64_t l_pac = 0;
    uint64_t n_sa = 0;
    uint32_t sa_shift = 0;
    uint64_t bwt_size = 0, primary = 0, L2[5] = {0, 0, 0, 0, 0};
    std::mutex mu;
    std::unordered_map<std::thread::id, smem_batch_t*> per_thread;
    // smem_gpu_collect_ex's batches by worker slot (the kt_for_batch tid):
    // kt_for_batch starts new threads for every chunk, so batches keyed by
    // thread would pile up; a slot's batch is reused by whichever thread holds
    // the slot next
    std::vector<smem_batch_t*> slots;
    // smem_gpu_seed_stream's worker batches, kept between calls: creating one
    // pins ~1 GB of host memory and allocates its device buffers
    std::vector<smem_batch_t*> stream_pool;
    // Admission (the role of the reference's HARP manager thread,
    // software/fastmap.c:320-429, which let one worker batch at a time onto
    // the FPGA and turned the others away): every entry point that runs work
    // on the device leases one of at most max_active stream pairs (a normal
    // and a low-priority stream, plus a third normal one for chains -> regions'
    // giant reads, smem_batch_chain2aln) for the duration of the call; more
    // concurrent calls wait for a pair.  So a device never carries more than
    // 3 x max_active streams, however many kt_for_batch workers share it.
    int max_active = 8;
    std::mutex adm_mu;
    std::condition_variable adm_cv;
    std::vector<std::pair<hipStream_t, hipStream_t>> pairs;
    std::vector<hipStream_t> thirds;  // pairs[k]'s third stream
    std::vector<int> free_pairs;
    int n_leased = 0;
    // a HIP runtime failure seen by any call: every later call fails at once
    // (SMEM_E_DEVICE) without touching the device, so the caller's reads take
    // its CPU path (software/bwt.c:686-717) and nothing more is enqueued on a
    // queue the runtime may have aborted
    std::atomic<int> faulted{0};
    char fault_msg[512] = {0};
    // background preparation started by smem_gpu_init_devices /
    // smem_gpu_reserve_slots: the densified SA (an event on init_st) and the
    // worker slots' pre-sized batches (a host thread)
    hipStream_t init_st = nullptr;
    hipEvent_t sa_ready = nullptr;
    uint64_t* d_sa_raw = nullptr;  // the .sa as uploaded (kept: the lookups use it until sa_ready has passed)
    uint64_t* d_link = nullptr;    // the densification's link scratch until sa_ready has passed (link_mu)
    std::mutex link_mu;
    uint32_t sa_shift_raw = 0;
    std::vector<std::shared_future<int>> reserve;  // smem_gpu_reserve_slots: one per slot
    // smem_gpu_init_devices_async: the upload running on a host thread; every
    // entry point that touches the device waits for it (gpu_wait)
    std::shared_future<int> ready;
    std::mutex ready_mu;  // ready is extended (gpu_chain) while other threads may wait on it
};

// the background upload of smem_gpu_init_devices_async has finished (its
// failure faulted the device, which gpu_check then reports)
static void gpu_wait(smem_gpu_t* g) {
    if (!g) return;
    std::shared_future<int> f;
    {
        std::lock_guard<std::mutex> lk(g->ready_mu);
        f = g->ready;
    }
    if (f.valid()) f.wait();
}

// scratch of the heavy-read path of chains -> regions
struct AlnHeavyBufs {
    DevBuf<int32_t> heavy, heavy2;
    DevBuf<uint64_t> hcnt, hoff, hscnt, hcnt2, hscnt2;
    // the giant split: read flags, the giants' walk counters, task list and lane queues, their
    // candidate index's segments
    DevBuf<uint8_t> rgiant, gtfail;
    DevBuf<uint32_t> gctr, gtorder, glq, chord_g;
    DevBuf<smem::RegTask> gtasks;
    DevBuf<uint64_t> ccnt_g, coff_g;
    DevBuf<uint8_t> ctmp_g;
    DevBuf<int64_t> span;
    DevBuf<uint64_t> ht;
    DevBuf<int32_t> rnext;
    DevBuf<smem::AlnReg> pre, pre_short, loc;
    DevBuf<uint8_t> short_ok, pre_ok, tmp;
    // the lane path (regions computed ahead one seed per lane)
    DevBuf<smem::RegTask> tasks, htasks;
    DevBuf<uint32_t> torder, lq, chain_read, swlist, htorder, hlq;
    DevBuf<uint8_t> tfail, sdec, htfail;
    // the heavy walk's candidate index
    DevBuf<uint64_t> ckey, ckey2, coff, ccnt;
    DevBuf<uint32_t> cval, cval2, cq, cpos_s, cpos_c, chord;
    DevBuf<int64_t> chmax, crb, cre;
    DevBuf<uint8_t> cmade, ctmp;
    DevBuf<uint2> crng;
    // f(buf) for every buffer (release, sizes)
    template <class F>
    void each(F&& f) {
        f(ckey); f(ckey2); f(coff); f(ccnt); f(cval); f(cval2); f(cq); f(cpos_s); f(cpos_c); f(chord); f(chmax);
        f(crb); f(cre); f(cmade); f(ctmp); f(crng); f(heavy); f(heavy2); f(hcnt2); f(hscnt2); f(rgiant); f(gtfail);
        f(gctr); f(gtorder); f(glq); f(chord_g); f(gtasks); f(ccnt_g); f(coff_g); f(ctmp_g); f(hcnt); f(hoff); f(hscnt); f(span); f(ht); f(rnext);
        f(pre); f(pre_short); f(loc); f(short_ok); f(pre_ok); f(tmp); f(tasks); f(torder); f(lq); f(tfail); f(sdec);
        f(chain_read); f(swlist); f(htasks); f(htorder); f(hlq); f(htfail);
    }
    void release() {
        each([](auto& x) { x.release(); });
    }
};

struct smem_batch {
    smem_gpu_t* g = nullptr;
    char* arena_dev = nullptr;   // the blocks a reserved slot's buffers are carved from (Arena)
    char* arena_host = nullptr;
    hipStream_t st = nullptr;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    // chains -> regions: the light reads' kernel runs on st2 beside the heavy
    // reads' kernels on st, joined by ev_join (created on first use)
    // (chaining: the heavy reads' second tier on st2, forked by ev_fork)
    hipStream_t st2 = nullptr;
    hipStream_t st3 = nullptr;  // chains -> regions: the giant reads' passes and walk (ev_giant joins them)
    hipEvent_t ev_join = nullptr, ev_fork = nullptr, ev_giant = nullptr;
    int max_reads = 0, max_len = 0;
    int read_len_max = 0;  // the longest read of the reads set (set_reads*)
    uint64_t max_bases = 0;
    uint32_t cap_intv = 0, cap_calls = 0, cap_list = 0;
    int lanes = 0;
    // staged reads
    int n_reads = 0;
    HostBuf<uint8_t> h_codes;
    HostBuf<uint64_t> h_offs;
    DevBuf<uint8_t> d_codes;
    DevBuf<uint64_t> d_offs;
    // seeding outputs
    DevBuf<Intv> d_out_intv;       // raw per-read lists
    DevBuf<CallRec> d_out_call;    // per-read list records
    DevBuf<uint32_t> d_n_intv, d_n_calls;
    DevBuf<int32_t> d_ctr;  // [0] head, [1] ovf_count, [2] ovf head, [3] ovf-ovf count
    DevBuf<int32_t> d_ovf_items, d_ovf_slot, d_ovf_items2;
    DevBuf<uint4> d_scratch;
    DevBuf<uint64_t> d_dbg;        // stamped variant only
    // overflow pass
    DevBuf<Intv> d_ovf_intv;
    DevBuf<CallRec> d_ovf_call;
    DevBuf<uint32_t> d_ovf_n_intv, d_ovf_n_calls;
    uint32_t ovf_cap_intv = 0, ovf_cap_calls = 0;
    // compaction
    DevBuf<uint64_t> d_sz_intv, d_sz_calls, d_intv_off, d_call_off;
    DevBuf<uint8_t> d_scan_tmp;
    DevBuf<Intv> d_flat_intv;
    DevBuf<uint32_t> d_flat_calls;
    HostBuf<int32_t> h_ctr;
    HostBuf<uint64_t> h_tot;
    // fetched results (packed: 16-B smem_pintv_t wire entries instead of h_intv)
    bool packed = false;
    DevBuf<uint4> d_pintv;
    HostBuf<uint4> h_pintv;
    HostBuf<Intv> h_intv;
    HostBuf<uint32_t> h_calls;
    HostBuf<uint64_t> h_intv_off, h_call_off;
    bool fetched = false, ran = false;
    uint64_t tot_intv = 0, tot_calls = 0;
    // bwt_sa of the seed occurrences (smem_batch_sa)
    DevBuf<uint64_t> d_occ_n, d_occ_off, d_sa_pos, d_kstart;
    DevBuf<uint8_t> d_sa_tmp;
    HostBuf<uint64_t> h_occ_off, h_sa_pos;
    bool sa_ran = false, sa_fetched = false;
    uint64_t tot_occ = 0;
    int sa_min_seed_len = 0;
    // chains (smem_batch_chain)
    DevBuf<smem::SeedRec> d_seed, d_out_seed;
    DevBuf<uint32_t> d_next, d_ord, d_ord2;
    DevBuf<smem::ChainRec> d_chn;
    DevBuf<smem::BNode> d_node;
    DevBuf<smem::FltRec> d_flt;
    DevBuf<uint64_t> d_n_out, d_ns_out, d_chain_off, d_seed_off;
    DevBuf<smem::OutChain> d_out_chain;
    DevBuf<uint32_t> d_heavy;
    HostBuf<uint64_t> h_chain_off;
    HostBuf<smem::OutChain> h_out_chain;
    HostBuf<smem::SeedRec> h_out_seed;
    bool chain_ran = false, chain_fetched = false, chain_filtered = false;
    uint64_t tot_chains = 0, tot_seeds = 0;
    // alignment regions (smem_batch_chain2aln)
    DevBuf<uint64_t> d_aln_srt, d_aln_nregs, d_aln_regoff;
    DevBuf<smem::AlnReg> d_aln_raw, d_aln_out;
    DevBuf<uint32_t> d_aln_ctr;
    AlnHeavyBufs aln_heavy;     // the heavy-read path's scratch
    HostBuf<uint64_t> h_aln_regoff;
    HostBuf<smem::AlnReg> h_aln_regs;
    bool aln_ran = false, aln_fetched = false;
    uint64_t tot_regs = 0;
    smem_batch_stats_t stats{};
};

// d(buf) for every device buffer of a batch, h(buf) for every pinned host one
template <class D, class H>
static void batch_bufs(smem_batch_t* b, D&& d, H&& h) {
    h(b->h_codes); h(b->h_offs); d(b->d_codes); d(b->d_offs);
    d(b->d_out_intv); d(b->d_out_call); d(b->d_n_intv); d(b->d_n_calls);
    d(b->d_ctr); d(b->d_ovf_items); d(b->d_ovf_slot); d(b->d_ovf_items2);
    d(b->d_scratch); d(b->d_dbg); d(b->d_ovf_intv); d(b->d_ovf_call); d(b->d_ovf_n_intv);
    d(b->d_ovf_n_calls); d(b->d_sz_intv); d(b->d_sz_calls); d(b->d_intv_off);
    d(b->d_call_off); d(b->d_scan_tmp); d(b->d_flat_intv); d(b->d_flat_calls);
    d(b->d_occ_n); d(b->d_occ_off); d(b->d_sa_pos); d(b->d_sa_tmp); d(b->d_kstart); h(b->h_occ_off); h(b->h_sa_pos);
    d(b->d_seed); d(b->d_out_seed); d(b->d_next); d(b->d_ord); d(b->d_ord2);
    d(b->d_chn); d(b->d_node); d(b->d_flt); d(b->d_n_out); d(b->d_ns_out);
    d(b->d_chain_off); d(b->d_seed_off); d(b->d_out_chain); d(b->d_heavy);
    h(b->h_chain_off); h(b->h_out_chain); h(b->h_out_seed);
    d(b->d_aln_srt); d(b->d_aln_nregs); d(b->d_aln_regoff); d(b->d_aln_raw);
    d(b->d_aln_out); d(b->d_aln_ctr); b->aln_heavy.each(d); h(b->h_aln_regoff); h(b->h_aln_regs);
    h(b->h_ctr); h(b->h_tot); h(b->h_intv); h(b->h_calls);
    d(b->d_pintv); h(b->h_pintv); h(b->h_intv_off); h(b->h_call_off);
}

static void guard_check(smem_batch_t* b, hipStream_t st, hipStream_t st2, hipStream_t st3) {
    if (st3) (void)hipStreamSynchronize(st3);
    (void)hipStreamSynchronize(st2);
    (void)hipStreamSynchronize(st);
    std::vector<uint8_t> h(GUARD_BYTES);
    int k = 0;
    batch_bufs(b, [&](auto& x) {
        if (x.p && x.own) {
            const char* tail = reinterpret_cast<const char*>(x.p) + x.n * sizeof(*x.p);
            if (hipMemcpy(h.data(), tail, GUARD_BYTES, hipMemcpyDeviceToHost) == hipSuccess) {
                size_t bad = 0, first = GUARD_BYTES;
                for (size_t i = 0; i < GUARD_BYTES; ++i)
                    if (h[i] != 0xA5) bad += 1, first = std::min(first, i);
                if (bad) {
                    fprintf(stderr, "[smem guard] batch %p (max_reads %d, max_len %d, ran %d/%d/%d/%d): buffer #%d of "
                            "%zu x %zu B written past its end: %zu guard bytes, the first at +%zu\n",
                            (void*)b, b->max_reads, b->max_len, (int)b->ran, (int)b->sa_ran, (int)b->chain_ran,
                            (int)b->aln_ran, k, x.n, sizeof(*x.p), bad, first);
                    (void)hipMemset(const_cast<char*>(tail), 0xA5, GUARD_BYTES);
                }
            }
        }
        ++k;
    }, [](auto&) {});
}

// ---- admission and the drain on the way out of every device call
static int gpu_check(smem_gpu_t* g) {
    if (!g->faulted.load()) return SMEM_OK;
    snprintf(g_err, sizeof(g_err), "device %d faulted earlier (%s): refused", g->device, g->fault_msg);
    return SMEM_E_DEVICE;
}

// One entry point's tenure on the device: refused at once on a faulted
// device, else it waits for one of the device's max_active stream pairs.  On
// the way out -- success, refusal or error alike -- both streams are
// synchronised before the pair goes back, so no kernel or copy of the call
// is still in flight (into the caller's or the library's host memory) once
// the caller resumes; a HIP runtime failure during the call marks the device
// faulted.
struct DeviceCall {
    smem_gpu_t* g;
    int pair = -1;
    hipStream_t st = nullptr, st2 = nullptr, st3 = nullptr;
    int rc = SMEM_OK;
    // third: the call needs the pair's third stream (chains -> regions), created on first use
    // -- made with every pair, the extra queue changed how the seeding workers' streams map to
    // the device's hardware queues and their launches overlapped less (21.8 -> 25.3 ms a step)
    explicit DeviceCall(smem_gpu_t* g_, bool third = false) : g(g_) {
        g_err[0] = 0;
        g_hip_fault = 0;
        const double t0 = now_s();
        gpu_wait(g);
        const double t1 = now_s();
        g_t_ready += t1 - t0;
        if ((rc = gpu_check(g))) return;
        hipError_t e = hipSetDevice(g->device);
        if (e != hipSuccess) {
            rc = fail(SMEM_E_DEVICE, "hipSetDevice", e);
            return;
        }
        std::unique_lock<std::mutex> lk(g->adm_mu);
        // leases are counted against max_active (a lowered limit holds even
        // when more pairs were made before it), pairs are reused first
        g->adm_cv.wait(lk, [&] {
            return g->n_leased < g->max_active && (!g->free_pairs.empty() || (int)g->pairs.size() < g->max_active);
        });
        g_t_admit += now_s() - t1;
        if (!g->free_pairs.empty()) {
            pair = g->free_pairs.back();
            g->free_pairs.pop_back();
        } else {
            hipStream_t a = nullptr, b = nullptr;
            int least = 0, greatest = 0;
            e = hipStreamCreateWithFlags(&a, hipStreamNonBlocking);
            if (e == hipSuccess) e = hipDeviceGetStreamPriorityRange(&least, &greatest);
            if (e == hipSuccess) e = hipStreamCreateWithPriority(&b, hipStreamNonBlocking, least);
            if (e != hipSuccess) {
                if (a) (void)hipStreamDestroy(a);
                rc = fail(SMEM_E_DEVICE, "admission: hipStreamCreate", e);
                g->adm_cv.notify_one();
                return;
            }
            g->pairs.emplace_back(a, b);
            g->thirds.push_back(nullptr);
            pair = (int)g->pairs.size() - 1;
        }
        if (third && !g->thirds[(size_t)pair]) {
            // the giant reads' passes, candidate index and walk (the alignment stage's
            // critical path), at the highest priority
            int least = 0, greatest = 0;
            hipStream_t c = nullptr;
            e = hipDeviceGetStreamPriorityRange(&least, &greatest);
            if (e == hipSuccess) e = hipStreamCreateWithPriority(&c, hipStreamNonBlocking, greatest);
            if (e != hipSuccess) {
                rc = fail(SMEM_E_DEVICE, "admission: hipStreamCreate (third)", e);
                g->free_pairs.push_back(pair);
                pair = -1;
                g->adm_cv.notify_one();
                return;
            }
            g->thirds[(size_t)pair] = c;
        }
        ++g->n_leased;
        st = g->pairs[(size_t)pair].first;
        st2 = g->pairs[(size_t)pair].second;
        st3 = g->thirds[(size_t)pair];
    }
    DeviceCall(const DeviceCall&) = delete;
    DeviceCall& operator=(const DeviceCall&) = delete;
    ~DeviceCall() {
        if (pair >= 0) {
            if (st3) (void)hipStreamSynchronize(st3);
            (void)hipStreamSynchronize(st2);
            (void)hipStreamSynchronize(st);
            std::lock_guard<std::mutex> lk(g->adm_mu);
            g->free_pairs.push_back(pair);
            --g->n_leased;
            g->adm_cv.notify_all();  // a waiter's predicate also depends on n_leased
        }
        if (g_hip_fault && !g->faulted.exchange(g_hip_fault)) {
            std::lock_guard<std::mutex> lk(g->adm_mu);
            snprintf(g->fault_msg, sizeof(g->fault_msg), "%s", g_err);
        }
    }
};

static void guard_check(smem_batch_t* b, hipStream_t st, hipStream_t st2, hipStream_t st3);

// a batch's call: the leased pair is the batch's st / st2 for its duration
struct BatchCall : DeviceCall {
    smem_batch_t* b;
    explicit BatchCall(smem_batch_t* b_, bool third = false) : DeviceCall(b_->g, third), b(b_) {
        if (rc == SMEM_OK) b->st = st, b->st2 = st2, b->st3 = st3;
    }
    ~BatchCall() {
        if (pair >= 0 && guard_on()) guard_check(b, st, st2, st3);
        b->st = b->st2 = b->st3 = nullptr;
    }
};

extern "C" {

#ifndef SMEM_SRC_HASH
#define SMEM_SRC_HASH "unknown"
#endif
const char* smem_gpu_build_id(void) { return SMEM_SRC_HASH; }
#ifndef SMEM_KERNEL_HASH
#define SMEM_KERNEL_HASH "unknown"
#endif
const char* smem_gpu_kernel_id(void) { return SMEM_KERNEL_HASH; }

const char* smem_strerror(int code) {
    if (g_err[0]) return g_err;
    switch (code) {
        case SMEM_OK: return "ok";
        case SMEM_E_ARG: return "bad argument";
        case SMEM_E_NOMEM: return "out of memory";
        case SMEM_E_IO: return "i/o error";
        case SMEM_E_DEVICE: return "HIP device error";
        case SMEM_E_CAPACITY: return "batch capacity exceeded";
        default: return "internal error";
    }
}

void smem_opt_default(smem_opt_t* o) {
    if (!o) return;
    o->min_seed_len = 19;   // software/bwamem.c:58
    o->split_factor = 1.5f; // software/bwamem.c:65
    o->split_width = 10;    // software/bwamem.c:59
    o->start_width = 1;     // software/bwamem.c:457 without MEM_F_NO_EXACT
}

int smem_gpu_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// a handle for `device` and the index's shape; gpu_open does the device work
static smem_gpu_t* gpu_handle(int device, uint64_t bwt_size, uint64_t primary, const uint64_t L2[5]) {
    smem_gpu_t* g = new (std::nothrow) smem_gpu_t();
    if (!g) return nullptr;
    g->device = device;
    if (const char* v = getenv("SMEM_GPU_MAX_ACTIVE")) g->max_active = std::max(1, std::min(256, atoi(v)));
    // the default seeding kernel for this handle (A/B: the same runs with another kernel);
    // a variant this build does not have is ignored
    if (const char* v = getenv("SMEM_GPU_SEED_VARIANT")) {
        const int sv = atoi(v);
        // (not the variants that need more than the Occ64 index -- 3 / 4 the reference layout,
        // 10 / 22 the Occ192 one, 23 the k-mer table, 9 / 25 the stamp buffer --: those only
        // through smem_gpu_set_kernel_variant / their own setup)
        if (sv > 0 && smem_seed_variant_built(sv) && sv != 3 && sv != 4 && sv != 9 && sv != 10 && sv != 22 &&
            sv != 23 && sv != 25)
            g->variant = sv;
    }
    // the CU count before any async init starts (smem_gpu_grid_reads may read it at once)
    if (hipDeviceGetAttribute(&g->n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) g->n_cu = 0;
    g->bwt_size = bwt_size;
    g->primary = primary;
    std::memcpy(g->L2, L2, sizeof(g->L2));
    return g;
}

// the index resident on g's device: upload, Occ64 re-layout (the device
// pointers stay null on failure)
static int gpu_open(smem_gpu_t* g, const uint32_t* bwt) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(SMEM_E_DEVICE, "smem_gpu_init: no HIP device");
    if (g->device < 0 || g->device >= n) return fail(SMEM_E_ARG, "smem_gpu_init: device out of range");
    HIP_TRY(hipSetDevice(g->device));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, g->device));
    if (g->n_cu <= 0) g->n_cu = prop.multiProcessorCount;  // (set by gpu_handle unless that query failed)
    const uint64_t bwt_size = g->bwt_size;
    // +16 words: a whole 64-B bucket can be loaded at the very end
    hipError_t e = hipMalloc(&g->d_bwt, (bwt_size + 16) * sizeof(uint32_t));
    if (e != hipSuccess) {
        g->d_bwt = nullptr;
        return fail(SMEM_E_NOMEM, "smem_gpu_init: hipMalloc(index)", e);
    }
    e = hipMemcpy(g->d_bwt, bwt, bwt_size * sizeof(uint32_t), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemset(g->d_bwt + bwt_size, 0, 16 * sizeof(uint32_t));
    if (e != hipSuccess) {
        (void)hipFree(g->d_bwt);
        g->d_bwt = nullptr;
        return fail(SMEM_E_DEVICE, "smem_gpu_init: upload", e);
    }
    // the Occ64 re-layout of the same index, built on the device
    const uint64_t n_ref = (bwt_size + 15) / 16;
    e = hipMalloc(&g->d_occ64, (n_ref * 16 + 16) * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemset(g->d_occ64 + n_ref * 16, 0, 16 * sizeof(uint32_t));
    if (e == hipSuccess) e = smem_launch_occ64(g->d_bwt, n_ref, g->d_occ64, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        (void)hipFree(g->d_bwt);
        if (g->d_occ64) (void)hipFree(g->d_occ64);
        g->d_bwt = nullptr;
        g->d_occ64 = nullptr;
        return fail(SMEM_E_DEVICE, "smem_gpu_init: Occ64 layout", e);
    }
#ifndef SMEM_AB_VARIANTS
    // only the A/B variants 3 / 4 read the reference layout: 3.1 GB of HBM
    // back at human size once Occ64 is built
    (void)hipFree(g->d_bwt);
    g->d_bwt = nullptr;
#endif
    // every kernel file's code object loaded now (~0.1 s, once per process
    // and device), beside bwa_idx_load's reading the .sa, not when the first
    // batch launches its kernels
    e = smem_preload_seed();
    if (e == hipSuccess) e = smem_preload_chain();
    if (e == hipSuccess) e = smem_preload_ksw();
    if (e == hipSuccess) e = smem_preload_aln();
    if (e != hipSuccess) return fail(SMEM_E_DEVICE, "smem_gpu_init: code objects", e);
    return SMEM_OK;
}

int smem_gpu_init(smem_gpu_t** out, int device, const uint32_t* bwt, uint64_t bwt_size, uint64_t primary,
                  const uint64_t L2[5]) {
    g_err[0] = 0;
    if (!out || !bwt || bwt_size < 16 || !L2) return fail(SMEM_E_ARG, "smem_gpu_init: bad index");
    // packed list entries hold SA coordinates in 34 bits
    if (L2[4] >= (1ull << 34) - 2) return fail(SMEM_E_ARG, "smem_gpu_init: seq_len >= 2^34 not supported");
    // Occ buckets are addressed as 32-bit byte offsets from the index base
    // (seq_len up to ~8.5 Gbp: both strands of a human genome are 6.2 Gbp)
    if ((bwt_size + 16) * sizeof(uint32_t) > (1ull << 32))
        return fail(SMEM_E_ARG, "smem_gpu_init: index larger than 4 GiB not supported");
    *out = nullptr;
    smem_gpu_t* g = gpu_handle(device, bwt_size, primary, L2);
    if (!g) return fail(SMEM_E_NOMEM, "smem_gpu_init");
    if (int rc = gpu_open(g, bwt)) {
        delete g;
        return rc;
    }
    *out = g;
    return SMEM_OK;
}

int smem_gpu_set_lanes_per_cu(smem_gpu_t* g, int lanes_per_cu) {
    if (!g) return SMEM_E_ARG;
    g->lanes_per_cu = lanes_per_cu > 0 ? std::max(64, lanes_per_cu / 64 * 64) : 0;
    return SMEM_OK;
}

int smem_gpu_set_kernel_variant(smem_gpu_t* g, int variant) {
    g_err[0] = 0;
    if (!g || !(variant == 0 || (variant >= 2 && variant <= 31) || (variant >= 40 && variant <= 62)))
        return fail(SMEM_E_ARG, "smem_gpu_set_kernel_variant");

    if (!smem_seed_variant_built(variant))
        return fail(SMEM_E_ARG, "smem_gpu_set_kernel_variant: A/B variant not in this build (make AB=1)");
    gpu_wait(g);
    if (int r = gpu_check(g)) return r;
    if ((variant == 10 || variant == 22) && !g->d_occ192) {
        // the Occ192 layout (variant 10 only), built from Occ64 on first use
        std::lock_guard<std::mutex> lk(g->mu);
        HIP_TRY(hipSetDevice(g->device));
        const uint64_t n_blocks = 2 * ((g->bwt_size + 15) / 16), n_lines = (n_blocks + 2) / 3;
        uint32_t* p = nullptr;
        HIP_TRY(hipMalloc(&p, (n_lines * 16 + 16) * sizeof(uint32_t)));
        hipError_t e = hipMemset(p + n_lines * 16, 0, 16 * sizeof(uint32_t));
        if (e == hipSuccess) e = smem_launch_occ192(g->d_occ64, n_blocks, p, nullptr);
        if (e == hipSuccess) e = hipDeviceSynchronize();
        if (e != hipSuccess) {
            (void)hipFree(p);
            return fail(SMEM_E_DEVICE, "smem_gpu_set_kernel_variant: Occ192 layout", e);
        }
        g->d_occ192 = p;
    }
    g->variant = variant == 0 ? kSeedDefault : variant;
    return SMEM_OK;
}

int smem_gpu_get_kernel_variant(const smem_gpu_t* g) { return g ? g->variant : SMEM_E_ARG; }

int smem_gpu_grid_reads(const smem_gpu_t* g) {
    if (!g) return SMEM_E_ARG;
    int n_cu = g->n_cu;
    if (n_cu <= 0 && hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, g->device) != hipSuccess)
        return SMEM_E_DEVICE;
    const int lpc = g->lanes_per_cu > 0 ? g->lanes_per_cu : seed_lanes_per_cu(g->variant);
    return (int)((int64_t)n_cu * lpc / 64 * seed_owners_per_wave(g->variant));
}

int smem_gpu_set_kmer_table(smem_gpu_t* g, int k) {
    g_err[0] = 0;
    if (!g || k < 0 || k > 15) return fail(SMEM_E_ARG, "smem_gpu_set_kmer_table: k must be 0..15");
    gpu_wait(g);
    if (int r = gpu_check(g)) return r;
    std::lock_guard<std::mutex> lk(g->mu);
    HIP_TRY(hipSetDevice(g->device));
    if (g->d_kt) {
        HIP_TRY(hipDeviceSynchronize());  // no batch may still read it
        (void)hipFree(g->d_kt);
        g->d_kt = nullptr;
        g->kt_k = 0;
    }
    if (k == 0) return SMEM_OK;
    const uint64_t n = ((1ull << (2 * (k + 1))) - 4) / 3;  // levels 1..k
    uint4* p = nullptr;
    hipError_t e = hipMalloc(&p, n * sizeof(uint4));
    if (e != hipSuccess) return fail(SMEM_E_NOMEM, "smem_gpu_set_kmer_table: hipMalloc", e);
    e = smem_launch_kmer_table(g->d_occ64, g->primary, g->L2, k, p, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        (void)hipFree(p);
        return fail(SMEM_E_DEVICE, "smem_gpu_set_kmer_table: build", e);
    }
    g->d_kt = p;
    g->kt_k = k;
    return SMEM_OK;
}

int smem_gpu_set_intv_cap(smem_gpu_t* g, int cap_per_read) {
    if (!g || cap_per_read < 0) return SMEM_E_ARG;
    g->intv_cap = cap_per_read;
    return SMEM_OK;
}

void smem_batch_destroy(smem_batch_t* b) {
    if (!b) return;
    // (every call drained its work before returning: nothing of this batch
    // is in flight, and its streams belong to the device's admission pool)
    (void)hipSetDevice(b->g->device);
    const double t0 = now_s();
    int nd = 0, nh = 0;
    batch_bufs(b, [&nd](auto& x) { nd += x.p && x.own; x.release(); }, [](auto&) {});
    const double t1 = now_s();
    batch_bufs(b, [](auto&) {}, [&nh](auto& x) { nh += x.p && x.own; x.release(); });
    if (b->arena_dev) (void)hipFree(b->arena_dev), ++nd;
    if (b->arena_host) (void)hipHostFree(b->arena_host), ++nh;
    g_rel_dev_ns += (int64_t)((t1 - t0) * 1e9);
    g_rel_host_ns += (int64_t)((now_s() - t1) * 1e9);
    g_rel_dev_n += nd;
    g_rel_host_n += nh;
    for (auto& ev : b->ev)
        if (ev) (void)hipEventDestroy(ev);
    if (b->ev_join) (void)hipEventDestroy(b->ev_join);
    if (b->ev_fork) (void)hipEventDestroy(b->ev_fork);
    if (b->ev_giant) (void)hipEventDestroy(b->ev_giant);
    delete b;
}

void smem_gpu_shutdown(smem_gpu_t* g) {
    if (!g) return;
    gpu_wait(g);
    for (auto& f : g->reserve)
        if (f.valid()) f.wait();
    (void)hipSetDevice(g->device);
    const double t0 = now_s();
    // the worker batches' device and pinned buffers, released on a few host
    // threads (unpinning host pages dominates)
    std::vector<smem_batch_t*> all;
    for (auto& kv : g->per_thread) all.push_back(kv.second);
    for (auto* b : g->slots) all.push_back(b);
    for (auto* b : g->stream_pool) all.push_back(b);
    g->per_thread.clear();
    g->slots.clear();
    g->stream_pool.clear();
    {
        const size_t nt = std::min<size_t>(all.size(), 8);
        std::vector<std::thread> th;
        for (size_t t = 0; t < nt; ++t)
            th.emplace_back([&all, t, nt]() {
                for (size_t k = t; k < all.size(); k += nt) smem_batch_destroy(all[k]);
            });
        for (auto& x : th) x.join();
    }
    const double t1 = now_s();
    if (g->d_bwt) (void)hipFree(g->d_bwt);
    if (g->d_occ64) (void)hipFree(g->d_occ64);
    if (g->d_occ192) (void)hipFree(g->d_occ192);
    if (g->d_kt) (void)hipFree(g->d_kt);
    if (g->init_st) (void)hipStreamSynchronize(g->init_st);
    if (g->d_link) (void)hipFree(g->d_link);
    if (g->d_sa) (void)hipFree(g->d_sa);
    if (g->d_sa_raw) (void)hipFree(g->d_sa_raw);
    if (g->d_pac) (void)hipFree(g->d_pac);
    for (auto& p : g->pairs) {
        (void)hipStreamDestroy(p.first);
        (void)hipStreamDestroy(p.second);
    }
    for (auto c : g->thirds)
        if (c) (void)hipStreamDestroy(c);
    if (g->sa_ready) (void)hipEventDestroy(g->sa_ready);
    if (g->init_st) (void)hipStreamDestroy(g->init_st);
    if (getenv("SMEM_GPU_TIMES"))
        fprintf(stderr, "[M::smem_gpu_shutdown] device %d: %zu batches released in %.4f s (thread-seconds: %lld device "
                "buffers %.4f, %lld pinned %.4f), index and streams in %.4f s\n", g->device, all.size(), t1 - t0,
                (long long)g_rel_dev_n.load(), g_rel_dev_ns.load() * 1e-9, (long long)g_rel_host_n.load(),
                g_rel_host_ns.load() * 1e-9, now_s() - t1);
    delete g;
}

int smem_batch_create(smem_gpu_t* g, int max_reads, uint64_t max_bases, int max_len, smem_batch_t** out) {
    g_err[0] = 0;
    if (!g || !out || max_reads <= 0 || max_len <= 0 || max_len > (1 << 24)) return fail(SMEM_E_ARG, "smem_batch_create");
    if (max_bases >= (1ull << 32) - 64) return fail(SMEM_E_ARG, "smem_batch_create: >= 2^32 bases per batch");
    *out = nullptr;
    gpu_wait(g);
    if (int r = gpu_check(g)) return r;
    HIP_TRY(hipSetDevice(g->device));
    smem_batch_t* b = new (std::nothrow) smem_batch_t();
    if (!b) return fail(SMEM_E_NOMEM, "smem_batch_create");
    b->g = g;
    b->max_reads = max_reads;
    b->max_bases = std::max<uint64_t>(max_bases, 1);
    b->max_len = max_len;
    // output capacity per read; reads that need more go through the overflow pass
    b->cap_intv = g->intv_cap > 0 ? (uint32_t)g->intv_cap : (uint32_t)std::max(32, max_len / 2 + 32);
    b->cap_calls = (uint32_t)(max_len / 4 + 16);  // ~6 lists per 150 bp read; more -> overflow pass
    b->cap_list = (uint32_t)max_len + 2;   // forward/backward lists hold <= len+1 intervals
    const int want_lanes = g->n_cu * (g->lanes_per_cu > 0 ? g->lanes_per_cu : seed_lanes_per_cu(g->variant));
    // a persistent grid of at most one lane per read: a batch under a full grid (the binding's
    // worker batches) runs beside the device's other admitted batches, which fill
    // the CUs its grid leaves, and each lane of the grid costs list-arena scratch (one arena per
    // owner, 2 x cap_list entries: 9 KB per read at 3 lanes a read and 256-bp slots).  Owners
    // (24 a wave) then take 2.7 reads each in turn.  batch_run_impl bounds each launch by
    // b->lanes, the lanes the scratch below was sized for, whatever variant is set later.
    const int read_lanes = (int)std::min<int64_t>((int64_t)max_reads + 255, INT32_MAX) / 256 * 256;
    b->lanes = std::max(256, std::min(want_lanes, read_lanes));
    int rc = SMEM_OK;
    hipError_t e = hipSuccess;
    for (int k = 0; k < 4 && e == hipSuccess; ++k) e = hipEventCreate(&b->ev[k]);
    const size_t R = (size_t)max_reads;
    if (e == hipSuccess) e = b->h_codes.ensure(b->max_bases);
    if (e == hipSuccess) e = b->h_offs.ensure(R + 1);
    if (e == hipSuccess) e = b->d_codes.ensure(b->max_bases + 32);  // 16-B query windows may read past the end
    if (e == hipSuccess) e = b->d_offs.ensure(R + 1);
    if (e == hipSuccess) e = b->d_out_intv.ensure(R * b->cap_intv);
    if (e == hipSuccess) e = b->d_out_call.ensure(R * b->cap_calls);
    if (e == hipSuccess) e = b->d_n_intv.ensure(R);
    if (e == hipSuccess) e = b->d_n_calls.ensure(R);
    if (e == hipSuccess) e = b->d_ctr.ensure(8);
    if (e == hipSuccess) e = b->d_ovf_items.ensure(R);
    if (e == hipSuccess) e = b->d_ovf_items2.ensure(R);
    if (e == hipSuccess) e = b->d_ovf_slot.ensure(R);
    if (e == hipSuccess) e = b->d_scratch.ensure(seed_arenas(g->variant, b->lanes) * 2 * b->cap_list);  // 2 packed lists
    if (e == hipSuccess) e = b->d_sz_intv.ensure(R);
    if (e == hipSuccess) e = b->d_sz_calls.ensure(R);
    if (e == hipSuccess) e = b->d_intv_off.ensure(R + 1);
    if (e == hipSuccess) e = b->d_call_off.ensure(R + 1);
    if (e == hipSuccess) e = b->h_ctr.ensure(8);
    if (e == hipSuccess) e = b->h_tot.ensure(16);  // [8, 16): run_aln's scalars
    if (e == hipSuccess) e = b->h_intv_off.ensure(R + 1);
    if (e == hipSuccess) e = b->h_call_off.ensure(R + 1);
    if (e == hipSuccess) {
        size_t tmp = 0;
        e = smem_launch_offsets(nullptr, nullptr, max_reads, nullptr, &tmp, b->st);
        if (e == hipSuccess) e = b->d_scan_tmp.ensure(tmp + 256);
    }
    if (e != hipSuccess) {
        rc = fail(SMEM_E_NOMEM, "smem_batch_create: allocation", e);
        smem_batch_destroy(b);
        return rc;
    }
    b->stats.block = 256;
    *out = b;
    return SMEM_OK;
}

// the staged reads host -> device, under the caller's BatchCall
static int upload_reads(smem_batch_t* b, int n_reads) {
    int ml = 0;
    for (int i = 0; i < n_reads; ++i) ml = std::max<int>(ml, (int)(b->h_offs.p[i + 1] - b->h_offs.p[i]));
    b->read_len_max = ml;
    b->ran = b->fetched = false;
    b->n_reads = 0;
    const uint64_t nb = b->h_offs.p[n_reads];
    HIP_TRY(hipMemcpyAsync(b->d_codes.p, b->h_codes.p, std::max<uint64_t>(nb, 1), hipMemcpyHostToDevice, b->st));
    HIP_TRY(hipMemcpyAsync(b->d_offs.p, b->h_offs.p, sizeof(uint64_t) * (n_reads + 1), hipMemcpyHostToDevice, b->st));
    INJECT(ST_UPLOAD);
    HIP_TRY(hipStreamSynchronize(b->st));
    b->n_reads = n_reads;
    return SMEM_OK;
}

int smem_batch_set_reads(smem_batch_t* b, int n_reads, const uint8_t* const* seq, const int* len) {
    g_err[0] = 0;
    if (!b || n_reads < 0 || (n_reads > 0 && (!seq || !len))) return fail(SMEM_E_ARG, "smem_batch_set_reads");
    if (n_reads > b->max_reads) return fail(SMEM_E_CAPACITY, "smem_batch_set_reads: too many reads");
    // (no copy from the staging buffers is in flight: every call drains its work)
    uint64_t o = 0;
    for (int i = 0; i < n_reads; ++i) {
        if (len[i] < 0 || len[i] > b->max_len) return fail(SMEM_E_CAPACITY, "smem_batch_set_reads: read too long");
        if (o + (uint64_t)len[i] > b->max_bases) return fail(SMEM_E_CAPACITY, "smem_batch_set_reads: too many bases");
        b->h_offs.p[i] = o;
        if (len[i]) std::memcpy(b->h_codes.p + o, seq[i], (size_t)len[i]);
        o += (uint64_t)len[i];
    }
    b->h_offs.p[n_reads] = o;
    BatchCall c(b);
    if (c.rc) return c.rc;
    return upload_reads(b, n_reads);
}

int smem_batch_set_reads_packed(smem_batch_t* b, int n_reads, const uint8_t* codes, const uint64_t* offsets) {
    g_err[0] = 0;
    if (!b || n_reads < 0 || !offsets || (n_reads > 0 && !codes)) return fail(SMEM_E_ARG, "smem_batch_set_reads_packed");
    if (n_reads > b->max_reads) return fail(SMEM_E_CAPACITY, "smem_batch_set_reads_packed: too many reads");
    const uint64_t o0 = offsets[0], nb = offsets[n_reads] - o0;
    if (nb > b->max_bases) return fail(SMEM_E_CAPACITY, "smem_batch_set_reads_packed: too many bases");
    for (int i = 0; i < n_reads; ++i) {
        const uint64_t l = offsets[i + 1] - offsets[i];
        if (offsets[i + 1] < offsets[i] || l > (uint64_t)b->max_len)
            return fail(SMEM_E_CAPACITY, "smem_batch_set_reads_packed: bad offsets / read too long");
        b->h_offs.p[i] = offsets[i] - o0;
    }
    b->h_offs.p[n_reads] = nb;
    if (nb) std::memcpy(b->h_codes.p, codes + o0, nb);
    BatchCall c(b);
    if (c.rc) return c.rc;
    return upload_reads(b, n_reads);
}

static void fill_params(smem_batch_t* b, const smem_opt_t* o, smem::SeedParams& P) {
    std::memset(&P, 0, sizeof(P));
    P.s_intv = b->d_sz_intv.p;   // per-read output sizes, written by the seeding kernel
    P.s_calls = b->d_sz_calls.p;
    P.bwt = b->g->d_bwt;
    P.occ64 = b->g->d_occ64;
    P.occ192 = b->g->d_occ192;
    P.kt = b->g->d_kt;
    P.kt_k = b->g->kt_k;
    P.primary = b->g->primary;
    std::memcpy(P.L2, b->g->L2, sizeof(P.L2));
    P.codes = b->d_codes.p;
    P.offs = b->d_offs.p;
    P.min_seed_len = o->min_seed_len;
    // exactly mem_insert_seed's expression (software/bwamem.c:456): int * float, + double, truncate
    P.split_len_init = (int)(o->min_seed_len * o->split_factor + .499);
    P.split_width = o->split_width;
    P.start_width = o->start_width;
    P.scratch = b->d_scratch.p;
    P.cap_list = b->cap_list;
    const char* dbg = getenv("SMEM_DEBUG_FLAGS");
    P.dbg = dbg ? atoi(dbg) : 0;
}

static int batch_run_impl(smem_batch_t* b, const smem_opt_t* opt) {
    smem_gpu_t* g = b->g;
    const int n = b->n_reads;
    b->fetched = false;
    b->sa_ran = false;
    b->sa_fetched = false;
    b->tot_occ = 0;
    b->chain_ran = b->chain_fetched = false;
    b->tot_chains = b->tot_seeds = 0;
    b->aln_ran = b->aln_fetched = false;
    b->tot_regs = 0;
    b->stats = smem_batch_stats_t{};
    b->stats.block = 256;
    smem::SeedParams P;
    fill_params(b, opt, P);
    // main pass: every read, output capacity cap_intv / cap_calls
    P.read_ids = nullptr;
    P.n_items = n;
    P.out_intv = b->d_out_intv.p;
    P.cap_intv = b->cap_intv;
    P.out_call = b->d_out_call.p;
    P.cap_calls = b->cap_calls;
    P.n_intv = b->d_n_intv.p;
    P.n_calls = b->d_n_calls.p;
    P.head = b->d_ctr.p + 0;
    P.ovf_count = b->d_ctr.p + 1;
    P.ovf_items = b->d_ovf_items.p;
    P.tspan = reinterpret_cast<uint64_t*>(b->d_ctr.p + 4);  // zeroed with the counters below
    const int lanes = std::min(b->lanes, std::max(256, (n * seed_lanes_per_read(g->variant) + 255) / 256 * 256));
    const int grid = lanes / 256;
    b->stats.grid = grid;
    // (a variant set after smem_batch_create may address more arenas than the batch was made for)
    HIP_TRY(b->d_scratch.ensure(seed_arenas(g->variant, b->lanes) * 2 * b->cap_list));
    P.scratch = b->d_scratch.p;
    HIP_TRY(hipMemsetAsync(b->d_ctr.p, 0, 8 * sizeof(int32_t), b->st));
    HIP_TRY(hipEventRecord(b->ev[0], b->st));
    if (g->variant == 23 && !g->d_kt) return fail(SMEM_E_ARG, "smem_batch_run: variant 23 needs smem_gpu_set_kmer_table");
    if (g->variant == 9 || g->variant == 25) {
        HIP_TRY(b->d_dbg.ensure((size_t)grid * 4 * 32));
        HIP_TRY(hipMemsetAsync(b->d_dbg.p, 0, (size_t)grid * 4 * 32 * sizeof(uint64_t), b->st));
        P.dbg_buf = b->d_dbg.p;
    }
    if (n > 0) HIP_TRY(smem_launch_seed(&P, grid, 256, g->variant, b->st));
    HIP_TRY(hipEventRecord(b->ev[1], b->st));
    HIP_TRY(hipMemcpyAsync(b->h_ctr.p, b->d_ctr.p, 8 * sizeof(int32_t), hipMemcpyDeviceToHost, b->st));
    HIP_TRY(hipStreamSynchronize(b->st));
    int n_ovf = b->h_ctr.p[1];
    b->stats.n_overflow = (uint32_t)n_ovf;
    if (n_ovf > 0) {
        // overflow pass: re-run the overflowed reads with larger capacities
        // until every one fits (bounded: results are finite)
        HIP_TRY(smem_launch_fill_i32(b->d_ovf_slot.p, -1, n, b->st));
        uint32_t cap_i = b->cap_intv * 4, cap_c = (uint32_t)b->max_len + 1;  // <= len lists per read
        for (int round = 0;; ++round) {
            if (round > 12) return fail(SMEM_E_INTERNAL, "smem_batch_run: overflow pass did not converge");
            HIP_TRY(b->d_ovf_intv.ensure((size_t)n_ovf * cap_i));
            HIP_TRY(b->d_ovf_call.ensure((size_t)n_ovf * cap_c));
            HIP_TRY(b->d_ovf_n_intv.ensure((size_t)n_ovf));
            HIP_TRY(b->d_ovf_n_calls.ensure((size_t)n_ovf));
            smem::SeedParams Q = P;
            Q.read_ids = b->d_ovf_items.p;  // overflowed read indices (main items == reads)
            Q.n_items = n_ovf;
            Q.out_intv = b->d_ovf_intv.p;
            Q.cap_intv = cap_i;
            Q.out_call = b->d_ovf_call.p;
            Q.cap_calls = cap_c;
            Q.n_intv = b->d_ovf_n_intv.p;
            Q.n_calls = b->d_ovf_n_calls.p;
            Q.head = b->d_ctr.p + 2;
            Q.ovf_count = b->d_ctr.p + 3;
            Q.ovf_items = b->d_ovf_items2.p;
            HIP_TRY(hipMemsetAsync(b->d_ctr.p + 2, 0, 2 * sizeof(int32_t), b->st));
            const int ql = std::min(b->lanes, (n_ovf * seed_lanes_per_read(g->variant) + 255) / 256 * 256);
            HIP_TRY(smem_launch_seed(&Q, std::max(1, ql / 256), 256, g->variant, b->st));
            HIP_TRY(hipMemcpyAsync(b->h_ctr.p, b->d_ctr.p, 8 * sizeof(int32_t), hipMemcpyDeviceToHost, b->st));
            HIP_TRY(hipStreamSynchronize(b->st));
            if (b->h_ctr.p[3] == 0) break;
            cap_i *= 4;
        }
        b->ovf_cap_intv = cap_i;
        b->ovf_cap_calls = cap_c;
        HIP_TRY(smem_launch_ovf_slot(b->d_ovf_items.p, n_ovf, b->d_ovf_slot.p, b->st));
    }
    // finalize: raw lists -> smem_next2 lists (scan of the sizes, write)
    HIP_TRY(hipEventRecord(b->ev[2], b->st));
    smem::FinalizeParams F;
    std::memset(&F, 0, sizeof(F));
    F.n = n;
    F.offs = b->d_offs.p;
    F.n_intv = b->d_n_intv.p;
    F.n_calls = b->d_n_calls.p;
    F.main_intv = b->d_out_intv.p;
    F.main_call = b->d_out_call.p;
    F.cap_intv = b->cap_intv;
    F.cap_calls = b->cap_calls;
    F.ovf_slot = b->d_ovf_slot.p;
    F.ovf_intv = b->d_ovf_intv.p;
    F.ovf_call = b->d_ovf_call.p;
    F.ovf_n_calls = b->d_ovf_n_calls.p;
    F.ovf_cap_intv = b->ovf_cap_intv;
    F.ovf_cap_calls = b->ovf_cap_calls;
    F.s_intv = b->d_sz_intv.p;
    F.s_calls = b->d_sz_calls.p;
    F.intv_off = b->d_intv_off.p;
    F.call_off = b->d_call_off.p;
    // (the sizes were written by the seeding kernel as each read completed)
    size_t tmp = b->d_scan_tmp.n;
    HIP_TRY(smem_launch_offsets(b->d_sz_intv.p, b->d_intv_off.p, n, b->d_scan_tmp.p, &tmp, b->st));
    HIP_TRY(smem_launch_offsets(b->d_sz_calls.p, b->d_call_off.p, n, b->d_scan_tmp.p, &tmp, b->st));
    HIP_TRY(hipMemcpyAsync(b->h_tot.p, b->d_intv_off.p + n, sizeof(uint64_t), hipMemcpyDeviceToHost, b->st));
    HIP_TRY(hipMemcpyAsync(b->h_tot.p + 1, b->d_call_off.p + n, sizeof(uint64_t), hipMemcpyDeviceToHost, b->st));
    HIP_TRY(hipStreamSynchronize(b->st));
    b->tot_intv = b->h_tot.p[0];
    b->tot_calls = b->h_tot.p[1];
    if (b->d_flat_intv.n < b->tot_intv || !b->d_flat_intv.p) {
        // grow with headroom so steady-state runs never reallocate
        HIP_TRY(b->d_flat_intv.ensure(std::max<size_t>(b->tot_intv + b->tot_intv / 4, (size_t)b->max_reads * 8)));
    }
    if (b->d_flat_calls.n < b->tot_calls || !b->d_flat_calls.p) {
        HIP_TRY(b->d_flat_calls.ensure(std::max<size_t>(b->tot_calls + b->tot_calls / 4, (size_t)b->max_reads * 4)));
    }
    F.flat_intv = b->d_flat_intv.p;
    F.flat_calls = b->d_flat_calls.p;
    HIP_TRY(smem_launch_finalize(&F, 1, b->st));
    HIP_TRY(hipEventRecord(b->ev[3], b->st));
    INJECT(ST_SEED);
    HIP_TRY(hipStreamSynchronize(b->st));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, b->ev[0], b->ev[1]));
    b->stats.kernel_ms = ms;
    HIP_TRY(hipEventElapsedTime(&ms, b->ev[2], b->ev[3]));
    b->stats.compact_ms = ms;
    b->stats.n_intv = b->tot_intv;
    b->stats.n_calls = b->tot_calls;
    {  // h_ctr was copied after the last seeding launch
        uint64_t sp[2];
        std::memcpy(sp, b->h_ctr.p + 4, sizeof(sp));
        b->stats.t_start = n > 0 ? ~sp[0] : 0;
        b->stats.t_end = n > 0 ? sp[1] : 0;
    }
    b->ran = true;
    return SMEM_OK;
}

int smem_batch_run(smem_batch_t* b, const smem_opt_t* opt) {
    g_err[0] = 0;
    if (!b || !opt) return fail(SMEM_E_ARG, "smem_batch_run");
    BatchCall c(b);
    if (c.rc) return c.rc;
    return batch_run_impl(b, opt);
}

// copy the outputs `mask` names (SMEM_FETCH_*) device -> pinned host memory
static int fetch_impl(smem_batch_t* b, int mask) {
    BatchCall call(b);
    if (call.rc) return call.rc;
    // views of an earlier fetch end here (its buffers may be regrown below)
    b->fetched = b->sa_fetched = b->chain_fetched = b->aln_fetched = false;
    const int n = b->n_reads;
    const bool f_intv = mask & SMEM_FETCH_INTV, f_sa = (mask & SMEM_FETCH_SA) && b->sa_ran;
    const bool f_chain = (mask & SMEM_FETCH_CHAINS) && b->chain_ran, f_aln = (mask & SMEM_FETCH_REGS) && b->aln_ran;
    // pinned result buffers grow with headroom: a streamed batch whose next
    // chunk holds a few more intervals must not re-pin a gigabyte
    if (!f_intv) {
    } else if (b->packed) {
        if (b->d_pintv.n < b->tot_intv || !b->d_pintv.p)
            HIP_TRY(b->d_pintv.ensure(std::max<uint64_t>(b->tot_intv + b->tot_intv / 4, 1)));
        if (b->h_pintv.n < b->tot_intv || !b->h_pintv.p)
            HIP_TRY(b->h_pintv.ensure(std::max<uint64_t>(b->tot_intv + b->tot_intv / 4, 1)));
    } else if (b->h_intv.n < b->tot_intv || !b->h_intv.p) {
        HIP_TRY(b->h_intv.ensure(std::max<uint64_t>(b->tot_intv + b->tot_intv / 4, 1)));
    }
    if (f_intv && (b->h_calls.n < b->tot_calls || !b->h_calls.p))
        HIP_TRY(b->h_calls.ensure(std::max<uint64_t>(b->tot_calls + b->tot_calls / 4, 1)));
    if (f_intv) {
        HIP_TRY(hipMemcpyAsync(b->h_intv_off.p, b->d_intv_off.p, sizeof(uint64_t) * (n + 1), hipMemcpyDeviceToHost, b->st));
        HIP_TRY(hipMemcpyAsync(b->h_call_off.p, b->d_call_off.p, sizeof(uint64_t) * (n + 1), hipMemcpyDeviceToHost, b->st));
    }
    if (!f_intv) {
    } else if (b->tot_intv && b->packed) {
        HIP_TRY(smem_launch_pack_intv(b->d_flat_intv.p, b->tot_intv, b->d_pintv.p, b->st));
        HIP_TRY(hipMemcpyAsync(b->h_pintv.p, b->d_pintv.p, sizeof(uint4) * b->tot_intv, hipMemcpyDeviceToHost, b->st));
    } else if (b->tot_intv) {
        HIP_TRY(hipMemcpyAsync(b->h_intv.p, b->d_flat_intv.p, sizeof(Intv) * b->tot_intv, hipMemcpyDeviceToHost, b->st));
    }
    if (f_intv && b->tot_calls)
        HIP_TRY(hipMemcpyAsync(b->h_calls.p, b->d_flat_calls.p, sizeof(uint32_t) * b->tot_calls, hipMemcpyDeviceToHost, b->st));
    if (f_sa) {
        HIP_TRY(b->h_occ_off.grow(b->tot_intv + 1));
        HIP_TRY(b->h_sa_pos.grow(b->tot_occ));
        HIP_TRY(hipMemcpyAsync(b->h_occ_off.p, b->d_occ_off.p, sizeof(uint64_t) * (b->tot_intv + 1),
                               hipMemcpyDeviceToHost, b->st));
        if (b->tot_occ)
            HIP_TRY(hipMemcpyAsync(b->h_sa_pos.p, b->d_sa_pos.p, sizeof(uint64_t) * b->tot_occ, hipMemcpyDeviceToHost,
                                   b->st));
    }
    if (f_chain) {
        HIP_TRY(b->h_chain_off.grow((uint64_t)n + 1));
        HIP_TRY(b->h_out_chain.grow(b->tot_chains));
        HIP_TRY(b->h_out_seed.grow(b->tot_seeds));
        HIP_TRY(hipMemcpyAsync(b->h_chain_off.p, b->d_chain_off.p, sizeof(uint64_t) * (n + 1), hipMemcpyDeviceToHost,
                               b->st));
        if (b->tot_chains)
            HIP_TRY(hipMemcpyAsync(b->h_out_chain.p, b->d_out_chain.p, sizeof(smem::OutChain) * b->tot_chains,
                                   hipMemcpyDeviceToHost, b->st));
        if (b->tot_seeds)
            HIP_TRY(hipMemcpyAsync(b->h_out_seed.p, b->d_out_seed.p, sizeof(smem::SeedRec) * b->tot_seeds,
                                   hipMemcpyDeviceToHost, b->st));
    }
    if (f_aln) {
        HIP_TRY(b->h_aln_regoff.grow((uint64_t)n + 1));
        HIP_TRY(b->h_aln_regs.grow(b->tot_regs));
        HIP_TRY(hipMemcpyAsync(b->h_aln_regoff.p, b->d_aln_regoff.p, sizeof(uint64_t) * (n + 1), hipMemcpyDeviceToHost,
                               b->st));
        if (b->tot_regs)
            HIP_TRY(hipMemcpyAsync(b->h_aln_regs.p, b->d_aln_out.p, sizeof(smem::AlnReg) * b->tot_regs,
                                   hipMemcpyDeviceToHost, b->st));
    }
    INJECT(ST_FETCH);
    HIP_TRY(hipStreamSynchronize(b->st));
    b->fetched = f_intv;
    b->sa_fetched = f_sa;
    b->chain_fetched = f_chain;
    b->aln_fetched = f_aln;
    return SMEM_OK;
}

int smem_batch_fetch(smem_batch_t* b) {
    g_err[0] = 0;
    if (!b || !b->ran) return fail(SMEM_E_ARG, "smem_batch_fetch: batch has not run");
    return fetch_impl(b, SMEM_FETCH_ALL);
}

int smem_batch_fetch_mask(smem_batch_t* b, int mask) {
    g_err[0] = 0;
    if (!b || !b->ran) return fail(SMEM_E_ARG, "smem_batch_fetch_mask: batch has not run");
    if (mask & ~SMEM_FETCH_ALL) return fail(SMEM_E_ARG, "smem_batch_fetch_mask: unknown bits");
    if (((mask & SMEM_FETCH_SA) && !b->sa_ran) || ((mask & SMEM_FETCH_CHAINS) && !b->chain_ran) ||
        ((mask & SMEM_FETCH_REGS) && !b->aln_ran))
        return fail(SMEM_E_ARG, "smem_batch_fetch_mask: a requested stage has not run on this batch");
    return fetch_impl(b, mask);
}


static int load_sa_impl(smem_gpu_t* g, const smem_sa_t* sa);
// The densification's link scratch (n_dense x 8 B: 12.4 GB at human size)
// comes from the device's default memory pool (hipMallocAsync on the init
// stream) and goes back to it with hipFreeAsync; the pool keeps freed memory
// reserved until trimmed.  Called once the densification has finished, so
// that smem_gpu_memory's budget is what stays allocated.
static hipError_t trim_default_pool(smem_gpu_t* g) {
    hipMemPool_t pool = nullptr;
    hipError_t e = hipDeviceGetDefaultMemPool(&pool, g->device);
    if (e == hipSuccess && pool) e = hipMemPoolTrimTo(pool, 0);
    return e;
}

// The link scratch of the default (SMEM_GPU_DENSIFY_POOL unset) densification is an allocation
// of its own, freed here once sa_ready has passed (hipFree waits for the device: once per
// handle).  The default pool is shared by every handle of the process: with eight handles on
// one GPU (the N = 8 fan-out rehearsed on one card) densifying side by side, a block one
// handle freed with hipFreeAsync came back to another while still in use and the dense SA
// came out wrong in ~15 % of runs (tools/flaky_probe.py, profiles/r06/multi_ctx).
static hipError_t release_link(smem_gpu_t* g, bool wait) {
    std::lock_guard<std::mutex> lk(g->link_mu);
    if (!g->d_link) return hipSuccess;
    if (wait) {
        hipError_t e = hipEventSynchronize(g->sa_ready);
        if (e != hipSuccess) return e;
    } else if (hipEventQuery(g->sa_ready) != hipSuccess) {
        (void)hipGetLastError();  // (not ready: a status, not an error of the caller's next call)
        return hipSuccess;
    }
    hipError_t e = hipFree(g->d_link);
    g->d_link = nullptr;
    return e;
}

// SMEM_GPU_SA_CHECK=1 (diagnostics, small indexes): every stored sample against the dense
// copy's row at the same position, after sa_ready; mismatches on stderr
static void sa_check(smem_gpu_t* g) {
    if (!getenv("SMEM_GPU_SA_CHECK") || !g->d_sa_raw || g->n_sa > (1ull << 28)) return;
    if (hipEventSynchronize(g->sa_ready) != hipSuccess) return;
    const uint64_t n_raw = (g->L2[4] >> g->sa_shift_raw) + 1, step = 1ull << (g->sa_shift_raw - g->sa_shift);
    std::vector<uint64_t> raw(n_raw), dense(g->n_sa);
    if (hipMemcpy(raw.data(), g->d_sa_raw, n_raw * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
    if (hipMemcpy(dense.data(), g->d_sa, g->n_sa * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
    uint64_t bad = 0, first = UINT64_MAX;
    for (uint64_t i = 0; i < n_raw && i * step < g->n_sa; ++i)
        if (raw[i] != dense[i * step]) bad += 1, first = std::min(first, i);
    uint64_t h = 1469598103934665603ull;  // FNV-1a over every dense row: equal across handles of one index
    for (uint64_t v : dense) h = (h ^ v) * 1099511628211ull;
    fprintf(stderr, "[M::sa_check] handle %p device %d: %llu of %llu stored samples differ from the dense SA "
            "(dense hash %016llx)%s\n", (void*)g, g->device, (unsigned long long)bad, (unsigned long long)n_raw,
            (unsigned long long)h, bad ? " (first at sample " : "");
    if (bad) fprintf(stderr, "[M::sa_check]   %llu)\n", (unsigned long long)first);
}

int smem_gpu_load_sa(smem_gpu_t* g, const smem_sa_t* sa) {
    g_err[0] = 0;
    gpu_wait(g);
    return load_sa_impl(g, sa);
}

static int load_sa_impl(smem_gpu_t* g, const smem_sa_t* sa) {
    if (!g || !sa || !sa->sa || sa->n_sa == 0 || sa->sa_intv == 0 || (sa->sa_intv & (sa->sa_intv - 1)))
        return fail(SMEM_E_ARG, "smem_gpu_load_sa: bad SA");
    if (sa->seq_len != g->L2[4] || sa->n_sa != (sa->seq_len + sa->sa_intv) / sa->sa_intv)
        return fail(SMEM_E_ARG, "smem_gpu_load_sa: SA does not belong to this index (seq_len)");
    if (sa->primary != g->primary) return fail(SMEM_E_ARG, "smem_gpu_load_sa: SA does not belong to this index (primary)");
    if (int r = gpu_check(g)) return r;
    HIP_TRY(hipSetDevice(g->device));
    if (g->d_sa || g->d_sa_raw) {
        // a reload: no batch may still read the old copy
        HIP_TRY(hipDeviceSynchronize());
        HIP_TRY(release_link(g, true));
        if (g->d_sa) (void)hipFree(g->d_sa);
        if (g->d_sa_raw) (void)hipFree(g->d_sa_raw);
        g->d_sa = g->d_sa_raw = nullptr;
    }
    // n_sa + 1 words: the zero pad of smem_sa_t (a 16-B load of the last sample stays in bounds)
    hipError_t e = hipMalloc(&g->d_sa, (sa->n_sa + 1) * sizeof(uint64_t));
    if (e != hipSuccess) return fail(SMEM_E_NOMEM, "smem_gpu_load_sa: hipMalloc", e);
    e = hipMemcpy(g->d_sa, sa->sa, sa->n_sa * sizeof(uint64_t), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemset(g->d_sa + sa->n_sa, 0, sizeof(uint64_t));
    if (e != hipSuccess) return fail(SMEM_E_DEVICE, "smem_gpu_load_sa: upload", e);
    g->n_sa = sa->n_sa;
    g->sa_shift = (uint32_t)__builtin_ctzll(sa->sa_intv);
    // a denser device copy (every SA_DENSE-th row, derived by LF walks from the
    // stored samples: same results, fewer steps per lookup); 8 B per
    // SA_DENSE symbols of HBM
    const uint32_t dshift = std::min<uint32_t>(g->sa_shift, SA_DENSE_SHIFT);
    if (dshift < g->sa_shift) {
        const uint64_t n_dense = (sa->seq_len + (1ull << dshift)) >> dshift;
        uint64_t* dense = nullptr;
        e = hipMalloc(&dense, (n_dense + 1) * sizeof(uint64_t));
        if (e != hipSuccess) return fail(SMEM_E_NOMEM, "smem_gpu_load_sa: hipMalloc(dense)", e);
        smem::SaParams S;
        std::memset(&S, 0, sizeof(S));
        S.occ64 = g->d_occ64;
        S.primary = g->primary;
        std::memcpy(S.L2, g->L2, sizeof(S.L2));
        S.sa = g->d_sa;
        S.sa_shift = g->sa_shift;
        // in the background, on the device's init stream: the caller goes on
        // (bwa mem reads its first chunk of reads, the first batches seed)
        // while the densification runs; until sa_ready has passed,
        // smem_batch_sa walks to the uploaded samples (kept until shutdown)
        if (!g->init_st) e = hipStreamCreateWithFlags(&g->init_st, hipStreamNonBlocking);
        if (e == hipSuccess && !g->sa_ready) e = hipEventCreateWithFlags(&g->sa_ready, hipEventDisableTiming);
        if (e == hipSuccess) e = hipMemsetAsync(dense + n_dense, 0, sizeof(uint64_t), g->init_st);
        // hop + chase passes (each BWT row stepped over once, ~0.2 s at human
        // size); SMEM_GPU_DENSIFY=walk: one full walk per dense row (the
        // round-3 kernel, ~0.7 s), kept for A/B
        const char* dv = getenv("SMEM_GPU_DENSIFY");
        if (e == hipSuccess && n_dense < (1ull << 32) && !(dv && !strcmp(dv, "walk"))) {
            uint64_t* link = nullptr;
            const char* pv = getenv("SMEM_GPU_DENSIFY_POOL");  // 1: the default pool (rounds 4-5; A/B only)
            const bool pool = pv && atoi(pv);
            e = pool ? hipMallocAsync((void**)&link, n_dense * sizeof(uint64_t), g->init_st)
                     : hipMalloc(&link, n_dense * sizeof(uint64_t));
            if (e == hipSuccess) {
                // the whole chip (capped at 4 blocks per CU so that the first
                // batches ran beside it, it finished later and they were no
                // faster: profiles/r04/e2e/probe_preload_densify_cap.log)
                e = smem_launch_sa_densify2(&S, dshift, n_dense, link, dense, 0u, g->init_st);
                if (pool) {
                    hipError_t f = hipFreeAsync(link, g->init_st);
                    if (e == hipSuccess) e = f;
                } else {
                    std::lock_guard<std::mutex> lk(g->link_mu);
                    g->d_link = link;  // release_link, once sa_ready has passed
                }
            }
        } else if (e == hipSuccess) {
            e = smem_launch_sa_densify(&S, dshift, n_dense, dense, g->init_st);
        }
        if (e == hipSuccess) e = hipEventRecord(g->sa_ready, g->init_st);
        if (e == hipSuccess && getenv("SMEM_GPU_TIMES"))  // diagnostics: when the device got there
            e = hipLaunchHostFunc(g->init_st, [](void* d) {
                fprintf(stderr, "[M::smem_gpu_load_sa] device %d: .sa densified at %.3f s\n", (int)(intptr_t)d,
                        now_s() - g_t_lib);
            }, (void*)(intptr_t)g->device);
        if (e == hipSuccess && getenv("SMEM_GPU_SYNC_INIT")) {
            e = hipStreamSynchronize(g->init_st);
            if (e == hipSuccess) e = trim_default_pool(g);
            if (e == hipSuccess) e = release_link(g, true);
        }
        if (e != hipSuccess) {
            (void)hipDeviceSynchronize();
            (void)hipFree(dense);
            return fail(SMEM_E_DEVICE, "smem_gpu_load_sa: densify", e);
        }
        g->d_sa_raw = g->d_sa;
        g->sa_shift_raw = g->sa_shift;
        g->d_sa = dense;
        g->n_sa = n_dense;
        g->sa_shift = dshift;
    }
    return SMEM_OK;
}

int smem_batch_sa(smem_batch_t* b, int min_seed_len, int max_occ) {
    g_err[0] = 0;
    if (!b || !b->ran) return fail(SMEM_E_ARG, "smem_batch_sa: batch has not run");
    smem_gpu_t* g = b->g;
    if (!g->d_sa) return fail(SMEM_E_ARG, "smem_batch_sa: no SA loaded (smem_gpu_load_sa)");
    if (max_occ < 0) return fail(SMEM_E_ARG, "smem_batch_sa: max_occ");
    BatchCall call(b);
    if (call.rc) return call.rc;
    b->sa_ran = b->chain_ran = b->aln_ran = false;
    b->sa_fetched = b->chain_fetched = b->aln_fetched = false;
    // the densified SA may still be in the making (smem_gpu_load_sa runs it
    // in the background): until its event has passed, the walk goes to the
    // stored samples instead (the same positions, sa_intv / D times the LF
    // steps), so no batch waits for it.  SMEM_GPU_SA_RAW=1: always the
    // stored samples (tests).
    const uint64_t* sa_rows = g->d_sa;
    uint32_t sa_shift = g->sa_shift;
    if (g->d_sa_raw) {
        const char* rv = getenv("SMEM_GPU_SA_RAW");
        hipError_t q = (rv && atoi(rv)) ? hipErrorNotReady : hipEventQuery(g->sa_ready);
        if (q == hipErrorNotReady) {
            (void)hipGetLastError();
            sa_rows = g->d_sa_raw;
            sa_shift = g->sa_shift_raw;
        } else if (q != hipSuccess) {
            return fail(SMEM_E_DEVICE, "smem_batch_sa: densification", q);
        } else if (g->d_link) {
            HIP_TRY(release_link(g, false));
        }
    }
    const uint64_t ni = b->tot_intv;
    if (ni >= (1ull << 31)) return fail(SMEM_E_CAPACITY, "smem_batch_sa: too many intervals");
    HIP_TRY(b->d_occ_n.grow(ni));
    HIP_TRY(b->d_occ_off.grow(ni + 1));
    size_t tmp = 0;
    HIP_TRY(smem_launch_offsets(nullptr, nullptr, (int)std::max<uint64_t>(ni, 1), nullptr, &tmp, b->st));
    HIP_TRY(b->d_sa_tmp.grow(tmp + 256));
    smem::SaParams S;
    std::memset(&S, 0, sizeof(S));
    S.occ64 = g->d_occ64;
    S.primary = g->primary;
    std::memcpy(S.L2, g->L2, sizeof(S.L2));
    S.sa = sa_rows;
    S.sa_shift = sa_shift;
    S.intv = b->d_flat_intv.p;
    S.n_intv = ni;
    S.min_seed_len = min_seed_len;
    S.max_occ = (uint64_t)max_occ;
    S.n_occ_intv = b->d_occ_n.p;
    S.occ_off = b->d_occ_off.p;
    HIP_TRY(hipEventRecord(b->ev[0], b->st));
    HIP_TRY(smem_launch_sa_count(&S, b->st));
    tmp = b->d_sa_tmp.n;
    HIP_TRY(smem_launch_offsets(b->d_occ_n.p, b->d_occ_off.p, (int)ni, b->d_sa_tmp.p, &tmp, b->st));
    HIP_TRY(hipMemcpyAsync(b->h_tot.p + 2, b->d_occ_off.p + ni, sizeof(uint64_t), hipMemcpyDeviceToHost, b->st));
    HIP_TRY(hipStreamSynchronize(b->st));
    b->tot_occ = b->h_tot.p[2];
    HIP_TRY(b->d_sa_pos.grow(std::max<uint64_t>(b->tot_occ, 1)));
    HIP_TRY(b->d_kstart.grow(b->tot_occ + 2));  // +2: the walk's aligned 16-B loads
    S.n_occ = b->tot_occ;
    S.pos = b->d_sa_pos.p;
    S.kstart = b->d_kstart.p;
    const int grid = std::max(1, (int)std::min<uint64_t>((uint64_t)g->n_cu * 8, (b->tot_occ + 255) / 256));
    HIP_TRY(smem_launch_sa_walk(&S, grid, b->st));
    HIP_TRY(hipEventRecord(b->ev[1], b->st));
    INJECT(ST_SA);
    HIP_TRY(hipStreamSynchronize(b->st));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, b->ev[0], b->ev[1]));
    b->stats.sa_ms = ms;
    b->stats.n_occ = b->tot_occ;
    b->sa_ran = true;
    b->sa_fetched = false;
    b->sa_min_seed_len = min_seed_len;
    b->chain_ran = b->chain_fetched = false;
    b->aln_ran = b->aln_fetched = false;
    return SMEM_OK;
}

void smem_chain_opt_default(smem_chain_opt_t* o) {
    if (!o) return;
    o->w = 100;                   // software/bwamem.c:53
    o->max_chain_gap = 10000;     // software/bwamem.c:61
    o->mask_level = 0.50f;        // software/bwamem.c:63
    o->chain_drop_ratio = 0.50f;  // software/bwamem.c:64
    o->filter = 1;                // mem_align1_core runs mem_chain_flt (software/bwamem.c:1449)
}

int smem_batch_chain(smem_batch_t* b, int64_t l_pac, const smem_chain_opt_t* opt) {
    g_err[0] = 0;
    if (!b || !b->sa_ran) return fail(SMEM_E_ARG, "smem_batch_chain: run smem_batch_sa first");
    if (!opt || l_pac < 0 || opt->w < 0) return fail(SMEM_E_ARG, "smem_batch_chain: bad options");
    if (b->tot_occ >= (1ull << 32) - 1) return fail(SMEM_E_CAPACITY, "smem_batch_chain: too many seed occurrences");
    BatchCall call(b);
    if (call.rc) return call.rc;
    b->chain_ran = b->aln_ran = false;
    b->chain_fetched = b->aln_fetched = false;
    const int n = b->n_reads;
    const uint64_t no = std::max<uint64_t>(b->tot_occ, 1);
    HIP_TRY(b->d_seed.grow(no));
    HIP_TRY(b->d_next.grow(no));
    HIP_TRY(b->d_chn.grow(no));
    HIP_TRY(b->d_node.grow(b->tot_occ / 7 + 3ull * (uint64_t)n + 8));
    HIP_TRY(b->d_ord.grow(no));
    HIP_TRY(b->d_ord2.grow(no));
    HIP_TRY(b->d_flt.grow(no));  // also the heavy path's per-seed codes
    HIP_TRY(b->d_n_out.grow(std::max(n, 1)));
    HIP_TRY(b->d_ns_out.grow(std::max(n, 1)));
    HIP_TRY(b->d_chain_off.grow(n + 1));
    HIP_TRY(b->d_seed_off.grow(n + 1));
    HIP_TRY(b->d_heavy.grow(2ull * (uint64_t)n + 4));
    size_t tmp = 0;
    HIP_TRY(smem_launch_offsets(nullptr, nullptr, std::max(n, 1), nullptr, &tmp, b->st));
    HIP_TRY(b->d_sa_tmp.grow(tmp + 256));
    smem::ChainParams P;
    std::memset(&P, 0, sizeof(P));
    P.intv = reinterpret_cast<const uint64_t*>(b->d_flat_intv.p);
    P.intv_off = b->d_intv_off.p;
    P.occ_off = b->d_occ_off.p;
    P.pos = b->d_sa_pos.p;
    P.n_reads = n;
    P.l_pac = l_pac;
    P.w = opt->w;
    P.max_chain_gap = opt->max_chain_gap;
    P.min_seed_len = b->sa_min_seed_len;
    P.filter = opt->filter ? 1 : 0;
    P.mask_level = opt->mask_level;
    P.drop_ratio = opt->chain_drop_ratio;
    P.seed = b->d_seed.p;
    P.next = b->d_next.p;
    P.chn = b->d_chn.p;
    P.node = b->d_node.p;
    P.ord = b->d_ord.p;
    P.ord2 = b->d_ord2.p;
    P.flt = b->d_flt.p;
    P.n_out = b->d_n_out.p;
    P.ns_out = b->d_ns_out.p;
    P.chain_off = b->d_chain_off.p;
    P.seed_off = b->d_seed_off.p;
    P.heavy_min = CHAIN_HEAVY_MIN;
    P.giant_min = CHAIN_GIANT_MIN;
    P.heavy_ctr = b->d_heavy.p;
    P.heavy = b->d_heavy.p + 4;
    P.lds_bytes = CHAIN_HEAVY_LDS;
    // test hooks: SMEM_CHAIN_LDS shrinks the heavy path's LDS (exercises its
    // HBM fallbacks), SMEM_CHAIN_HEAVY_MIN moves the lane/wave split
    if (const char* v = getenv("SMEM_CHAIN_LDS")) P.lds_bytes = (uint32_t)std::max(1024, atoi(v));
    if (const char* v = getenv("SMEM_CHAIN_HEAVY_MIN")) P.heavy_min = (uint32_t)std::max(0, atoi(v));
    if (const char* v = getenv("SMEM_CHAIN_GIANT_MIN")) P.giant_min = (uint32_t)std::max(0, atoi(v));
    P.cluster = getenv("SMEM_CHAIN_TREE_ONLY") ? 0 : 1;
    P.wave_sort = getenv("SMEM_CHAIN_SERIAL_SORT") ? 0 : 1;
    P.sort_lane_max = 128;  // r7h: 128 vs 256, human-like 22.5-22.7 vs 22.5-23.4 ms, uniform 14.2-14.3 vs 14.3-14.5
    P.drop_blocked = getenv("SMEM_CHAIN_DROP_PRUNED") ? 0 : 1;
    // the replay's chain-record cache and the wave-batched big clusters are off by default: both
    // measured slower (filtered, 1M reads: uniform 14.7 -> 16.1-16.2 ms with both, human-like 26.2 ->
    // 26.6-27.4; each alone between; profiles/r05/chain_ab.txt).  SMEM_CHAIN_REPLAY_CACHE=1 and
    // SMEM_CHAIN_WAVE_MIN=<seeds> turn them on (tests/test_gpu_chain.py keeps them bit-exact)
    P.replay_cache = getenv("SMEM_CHAIN_REPLAY_CACHE") && atoi(getenv("SMEM_CHAIN_REPLAY_CACHE")) == 1 ? 1 : 0;
    P.wave_min = 0xFFFFFFFFu;  // SMEM_CHAIN_WAVE_MIN: clusters of more seeds by the whole wave
    P.sort_count = getenv("SMEM_CHAIN_SORT_COUNT") && atoi(getenv("SMEM_CHAIN_SORT_COUNT")) == 0 ? 0 : 1;
    P.giant_order = getenv("SMEM_CHAIN_GIANT_ORDER") ? std::min(2, std::max(0, atoi(getenv("SMEM_CHAIN_GIANT_ORDER")))) : 0;
    P.giant_waves = getenv("SMEM_CHAIN_GIANT_WAVES") ? (uint32_t)std::max(1, atoi(getenv("SMEM_CHAIN_GIANT_WAVES"))) : 0u;
    P.dbg_lo = getenv("SMEM_CHAIN_DBG_LO") ? (uint32_t)strtoul(getenv("SMEM_CHAIN_DBG_LO"), nullptr, 10) : 0u;
    if (const char* v = getenv("SMEM_CHAIN_WAVE_MIN")) P.wave_min = (uint32_t)strtoul(v, nullptr, 10);
    if (const char* v = getenv("SMEM_CHAIN_SORT_LANE_MAX")) P.sort_lane_max = (uint32_t)std::max(17, atoi(v));
    if (getenv("SMEM_CHAIN_DBG")) {
        HIP_TRY(b->d_dbg.ensure(256 * 32));
        HIP_TRY(hipMemsetAsync(b->d_dbg.p, 0, 256 * 32 * sizeof(uint64_t), b->st));
        P.dbg = b->d_dbg.p;
    }
    // the heavy reads' second tier beside the giants (SMEM_CHAIN_STREAMS=1:
    // one launch of both on the batch's stream; SMEM_CHAIN_LDS_REST: its LDS)
    P.lds_rest = CHAIN_REST_LDS;
    if (const char* v = getenv("SMEM_CHAIN_LDS_REST")) P.lds_rest = (uint32_t)std::max(1024, atoi(v));
    const bool two = !(getenv("SMEM_CHAIN_STREAMS") && atoi(getenv("SMEM_CHAIN_STREAMS")) == 1);
    if (two && !b->ev_fork) HIP_TRY(hipEventCreateWithFlags(&b->ev_fork, hipEventDisableTiming));
    if (two && !b->ev_join) HIP_TRY(hipEventCreateWithFlags(&b->ev_join, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(b->ev[0], b->st));
    HIP_TRY(smem_launch_chain_build(&P, b->g->n_cu, b->st, two ? b->st2 : nullptr, b->ev_fork, b->ev_join));
    tmp = b->d_sa_tmp.n;
    HIP_TRY(smem_launch_offsets(b->d_n_out.p, b->d_chain_off.p, n, b->d_sa_tmp.p, &tmp, b->st));
    tmp = b->d_sa_tmp.n;
    HIP_TRY(smem_launch_offsets(b->d_ns_out.p, b->d_seed_off.p, n, b->d_sa_tmp.p, &tmp, b->st));
    HIP_TRY(hipMemcpyAsync(b->h_tot.p + 3, b->d_chain_off.p + n, sizeof(uint64_t), hipMemcpyDeviceToHost, b->st));
    HIP_TRY(hipMemcpyAsync(b->h_tot.p + 4, b->d_seed_off.p + n, sizeof(uint64_t), hipMemcpyDeviceToHost, b->st));
    HIP_TRY(hipStreamSynchronize(b->st));
    b->tot_chains = b->h_tot.p[3];
    b->tot_seeds = b->h_tot.p[4];
    HIP_TRY(b->d_out_chain.grow(std::max<uint64_t>(b->tot_chains, 1)));
    HIP_TRY(b->d_out_seed.grow(std::max<uint64_t>(b->tot_seeds, 1)));
    P.out_chain = b->d_out_chain.p;
    P.out_seed = b->d_out_seed.p;
    HIP_TRY(smem_launch_chain_write(&P, b->g->n_cu, b->st));
    HIP_TRY(hipEventRecord(b->ev[1], b->st));
    INJECT(ST_CHAIN);
    HIP_TRY(hipStreamSynchronize(b->st));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, b->ev[0], b->ev[1]));
    b->stats.chain_ms = ms;
    b->stats.n_chains = b->tot_chains;
    b->chain_ran = true;
    b->chain_fetched = false;
    b->chain_filtered = opt->filter != 0;
    b->aln_ran = b->aln_fetched = false;
    return SMEM_OK;
}

int smem_batch_chain_results(const smem_batch_t* b, const smem_chain_t** chains, const uint64_t** chain_off,
                             const smem_seed_t** seeds, uint64_t* n_chains, uint64_t* n_seeds) {
    if (!b || !b->chain_fetched) return SMEM_E_ARG;
    if (chains) *chains = reinterpret_cast<const smem_chain_t*>(b->h_out_chain.p);
    if (chain_off) *chain_off = b->h_chain_off.p;
    if (seeds) *seeds = reinterpret_cast<const smem_seed_t*>(b->h_out_seed.p);
    if (n_chains) *n_chains = b->tot_chains;
    if (n_seeds) *n_seeds = b->tot_seeds;
    return SMEM_OK;
}

int smem_batch_sa_results(const smem_batch_t* b, const uint64_t** pos, const uint64_t** occ_off, uint64_t* n_occ) {
    if (!b || !b->sa_fetched) return SMEM_E_ARG;
    if (pos) *pos = b->h_sa_pos.p;
    if (occ_off) *occ_off = b->h_occ_off.p;
    if (n_occ) *n_occ = b->tot_occ;
    return SMEM_OK;
}

int smem_batch_read(const smem_batch_t* b, int i, const smem_intv_t** intv, int* n_intv, const uint32_t** call_n,
                    int* n_calls) {
    if (!b || !b->fetched || b->packed || i < 0 || i >= b->n_reads) return SMEM_E_ARG;
    const uint64_t o = b->h_intv_off.p[i], co = b->h_call_off.p[i];
    if (intv) *intv = reinterpret_cast<const smem_intv_t*>(b->h_intv.p + o);
    if (n_intv) *n_intv = (int)(b->h_intv_off.p[i + 1] - o);
    if (call_n) *call_n = b->h_calls.p + co;
    if (n_calls) *n_calls = (int)(b->h_call_off.p[i + 1] - co);
    return SMEM_OK;
}

int smem_batch_results_packed(const smem_batch_t* b, const smem_pintv_t** pintv, const uint64_t** intv_off,
                              const uint32_t** call_n, const uint64_t** call_off) {
    if (!b || !b->fetched || !b->packed) return SMEM_E_ARG;
    if (pintv) *pintv = reinterpret_cast<const smem_pintv_t*>(b->h_pintv.p);
    if (intv_off) *intv_off = b->h_intv_off.p;
    if (call_n) *call_n = b->h_calls.p;
    if (call_off) *call_off = b->h_call_off.p;
    return SMEM_OK;
}

int smem_batch_results(const smem_batch_t* b, const smem_intv_t** intv, const uint64_t** intv_off,
                       const uint32_t** call_n, const uint64_t** call_off) {
    if (!b || !b->fetched || b->packed) return SMEM_E_ARG;
    if (intv) *intv = reinterpret_cast<const smem_intv_t*>(b->h_intv.p);
    if (intv_off) *intv_off = b->h_intv_off.p;
    if (call_n) *call_n = b->h_calls.p;
    if (call_off) *call_off = b->h_call_off.p;
    return SMEM_OK;
}

int smem_batch_debug(const smem_batch_t* b, uint64_t* out, uint64_t n_words) {
    if (!b || !out || !b->d_dbg.p) return SMEM_E_ARG;
    const uint64_t n = std::min<uint64_t>(n_words, b->d_dbg.n);
    if (hipMemcpy(out, b->d_dbg.p, n * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) return SMEM_E_DEVICE;
    return (int)n;
}

void smem_ksw_opt_default(smem_ksw_opt_t* o) {
    if (!o) return;
    std::memset(o, 0, sizeof(*o));
    // bwa_fill_scmat(1, 4) (software/bwa.c:84-93), gaps of mem_opt_init (software/bwamem.c:50-52)
    for (int i = 0; i < 4; ++i) {
        for (int j = 0; j < 4; ++j) o->mat[i * 5 + j] = (int8_t)(i == j ? 1 : -4);
        o->mat[i * 5 + 4] = -1;
    }
    for (int j = 0; j < 5; ++j) o->mat[20 + j] = -1;
    o->o_del = o->o_ins = 6;
    o->e_del = o->e_ins = 1;
}

static_assert(sizeof(smem_ksw_task_t) == sizeof(smem::KswTask), "task layout");
static_assert(sizeof(smem_ksw_result_t) == sizeof(smem::KswResult), "result layout");

int smem_ksw_extend(smem_gpu_t* g, int n, const smem_ksw_task_t* tasks, const uint8_t* q, uint64_t q_bytes,
                    const uint8_t* t, uint64_t t_bytes, const smem_ksw_opt_t* opt, smem_ksw_result_t* out,
                    double* kernel_ms) {
    g_err[0] = 0;
    if (!g || n < 0 || !opt || (n > 0 && (!tasks || !out))) return fail(SMEM_E_ARG, "smem_ksw_extend: bad arguments");
    if (opt->e_del < 1 || opt->e_ins < 1 || opt->o_del < 0 || opt->o_ins < 0)
        return fail(SMEM_E_ARG, "smem_ksw_extend: gap penalties need e >= 1, o >= 0");
    for (int i = 0; i < n; ++i) {
        const smem_ksw_task_t& k = tasks[i];
        if (k.qlen < 1 || k.qlen > 64 * smem::KSW_COLS_PER_LANE - 1 || k.tlen < 0 || k.q_off + (uint64_t)k.qlen > q_bytes ||
            k.t_off + (uint64_t)k.tlen > t_bytes)
            return fail(SMEM_E_ARG, "smem_ksw_extend: task outside 1 <= qlen <= 255 or its pools");
    }
    if (kernel_ms) *kernel_ms = 0.0;
    if (n == 0) return SMEM_OK;
    DevBuf<smem::KswTask> dt;
    DevBuf<smem::KswResult> dr;
    DevBuf<uint8_t> dq, dtg, dsc;
    hipEvent_t ev[2] = {nullptr, nullptr};
    struct Guard {
        DevBuf<smem::KswTask>& a; DevBuf<smem::KswResult>& b; DevBuf<uint8_t>& c; DevBuf<uint8_t>& d;
        DevBuf<uint8_t>& f; hipEvent_t* e;
        ~Guard() {
            a.release(); b.release(); c.release(); d.release(); f.release();
            if (e[0]) (void)hipEventDestroy(e[0]);
            if (e[1]) (void)hipEventDestroy(e[1]);
        }
    } guard{dt, dr, dq, dtg, dsc, ev};
    DeviceCall call(g);  // (declared after the buffers: drained before they are freed)
    if (call.rc) return call.rc;
    const hipStream_t st = call.st;
    HIP_TRY(hipEventCreate(&ev[0]));
    HIP_TRY(hipEventCreate(&ev[1]));
    HIP_TRY(dt.ensure(n));
    HIP_TRY(dr.ensure(n));
    HIP_TRY(dq.ensure(q_bytes + 64));
    HIP_TRY(dtg.ensure(t_bytes + 64));
    // SMEM_KSW_LANE=1: one problem per lane (kswl::lane_engine), tiers by query length
    const char* lane_e = getenv("SMEM_KSW_LANE");
    const bool lane = lane_e && atoi(lane_e);
    // the one-wave-per-problem kernel takes the problems in query-length order (a stable
    // counting sort on the host; the results are put back in the caller's order below):
    // neighbouring waves then run the same column tier, 5.98 -> 5.29 ms on 200k problems
    // (profiles/r05/ksw/ksw_ab_r6j.txt, wave_sorted); SMEM_KSW_SORT=0 keeps the caller's order
    const char* sort_e = getenv("SMEM_KSW_SORT");
    const bool sorted = !lane && !(sort_e && atoi(sort_e) == 0);
    std::vector<uint32_t> order;
    std::vector<smem::KswTask> stask;
    if (sorted) {
        uint32_t cnt[257] = {0};
        for (int i = 0; i < n; ++i) ++cnt[tasks[i].qlen + 1];
        for (int k = 1; k < 257; ++k) cnt[k] += cnt[k - 1];
        order.resize(n);
        stask.resize(n);
        for (int i = 0; i < n; ++i) order[cnt[tasks[i].qlen]++] = (uint32_t)i;
        for (int i = 0; i < n; ++i) std::memcpy(&stask[i], &tasks[order[i]], sizeof(smem::KswTask));
    }
    HIP_TRY(hipMemcpyAsync(dt.p, sorted ? (const void*)stask.data() : (const void*)tasks, sizeof(smem::KswTask) * n,
                           hipMemcpyHostToDevice, st));
    if (q_bytes) HIP_TRY(hipMemcpyAsync(dq.p, q, q_bytes, hipMemcpyHostToDevice, st));
    if (t_bytes) HIP_TRY(hipMemcpyAsync(dtg.p, t, t_bytes, hipMemcpyHostToDevice, st));
    smem::KswParams K;
    std::memset(&K, 0, sizeof(K));
    K.task = dt.p;
    K.n = n;
    K.q = dq.p;
    K.t = dtg.p;
    std::memcpy(K.mat, opt->mat, 25);
    K.o_del = opt->o_del;
    K.e_del = opt->e_del;
    K.o_ins = opt->o_ins;
    K.e_ins = opt->e_ins;
    K.out = dr.p;
    if (lane) HIP_TRY(dsc.ensure(smem_ksw_lane_scratch(n)));
    HIP_TRY(hipEventRecord(ev[0], st));
    if (lane) HIP_TRY(smem_launch_ksw_lane(&K, dsc.p, g->n_cu, st));
    else HIP_TRY(smem_launch_ksw(&K, g->n_cu, st));
    HIP_TRY(hipEventRecord(ev[1], st));
    std::vector<smem_ksw_result_t> sres;
    if (sorted) sres.resize(n);
    HIP_TRY(hipMemcpyAsync(sorted ? (void*)sres.data() : (void*)out, dr.p, sizeof(smem::KswResult) * n,
                           hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    for (int i = 0; sorted && i < n; ++i) out[order[i]] = sres[i];
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, ev[0], ev[1]));
    if (kernel_ms) *kernel_ms = ms;
    return SMEM_OK;
}

static_assert(sizeof(smem_ksw_atask_t) == sizeof(smem::KswATask), "align task layout");
static_assert(sizeof(smem_ksw_aresult_t) == sizeof(smem::KswAResult), "align result layout");

int smem_ksw_align2(smem_gpu_t* g, int n, const smem_ksw_atask_t* tasks, const uint8_t* q, uint64_t q_bytes,
                    const uint8_t* t, uint64_t t_bytes, const smem_ksw_opt_t* opt, smem_ksw_aresult_t* out,
                    double* kernel_ms) {
    g_err[0] = 0;
    if (!g || n < 0 || !opt || (n > 0 && (!tasks || !out))) return fail(SMEM_E_ARG, "smem_ksw_align2: bad arguments");
    if (opt->e_del < 1 || opt->e_ins < 1 || opt->o_del < 0 || opt->o_ins < 0)
        return fail(SMEM_E_ARG, "smem_ksw_align2: gap penalties need e >= 1, o >= 0");
    for (int i = 0; i < n; ++i) {
        const smem_ksw_atask_t& k = tasks[i];
        if (k.qlen < 1 || k.qlen > 256 || k.tlen < 0 || k.tlen > 256 || k.q_off + (uint64_t)k.qlen > q_bytes ||
            k.t_off + (uint64_t)k.tlen > t_bytes)
            return fail(SMEM_E_ARG, "smem_ksw_align2: task outside 1 <= qlen <= 256, tlen <= 256 or its pools");
        // a byte-scored problem must not overflow 255 from below the bias (ksw_align2's callers size
        // XBYTE for that; a saturated u8 score is returned as 255, as ksw_u8 does)
    }
    for (uint64_t k = 0; k < q_bytes; ++k)
        if (q[k] > 4) return fail(SMEM_E_ARG, "smem_ksw_align2: query code > 4");
    if (kernel_ms) *kernel_ms = 0.0;
    if (n == 0) return SMEM_OK;
    DevBuf<smem::KswATask> dt;
    DevBuf<smem::KswAResult> dr;
    DevBuf<uint8_t> dq, dtg;
    hipEvent_t ev[2] = {nullptr, nullptr};
    struct Guard {
        DevBuf<smem::KswATask>& a; DevBuf<smem::KswAResult>& b; DevBuf<uint8_t>& c; DevBuf<uint8_t>& d;
        hipEvent_t* e;
        ~Guard() {
            a.release(); b.release(); c.release(); d.release();
            if (e[0]) (void)hipEventDestroy(e[0]);
            if (e[1]) (void)hipEventDestroy(e[1]);
        }
    } guard{dt, dr, dq, dtg, ev};
    DeviceCall call(g);  // (declared after the buffers: drained before they are freed)
    if (call.rc) return call.rc;
    const hipStream_t st = call.st;
    HIP_TRY(hipEventCreate(&ev[0]));
    HIP_TRY(hipEventCreate(&ev[1]));
    HIP_TRY(dt.ensure(n));
    HIP_TRY(dr.ensure(n));
    HIP_TRY(dq.ensure(q_bytes + 64));
    HIP_TRY(dtg.ensure(t_bytes + 64));
    HIP_TRY(hipMemcpyAsync(dt.p, tasks, sizeof(smem::KswATask) * n, hipMemcpyHostToDevice, st));
    if (q_bytes) HIP_TRY(hipMemcpyAsync(dq.p, q, q_bytes, hipMemcpyHostToDevice, st));
    if (t_bytes) HIP_TRY(hipMemcpyAsync(dtg.p, t, t_bytes, hipMemcpyHostToDevice, st));
    smem::KswAParams K;
    std::memset(&K, 0, sizeof(K));
    K.task = dt.p, K.n = n, K.q = dq.p, K.t = dtg.p, K.out = dr.p;
    std::memcpy(K.mat, opt->mat, 25);
    K.o_del = opt->o_del, K.e_del = opt->e_del, K.o_ins = opt->o_ins, K.e_ins = opt->e_ins;
    {  // ksw_qinit's bias and largest score (software/ksw.c:78-85)
        uint8_t sh = 127, md = 0;
        for (int k = 0; k < 25; ++k) {
            if (opt->mat[k] < (int8_t)sh) sh = (uint8_t)opt->mat[k];
            if (opt->mat[k] > (int8_t)md) md = (uint8_t)opt->mat[k];
        }
        K.top = md, K.shift = (uint8_t)(256 - sh);
    }
    HIP_TRY(hipEventRecord(ev[0], st));
    HIP_TRY(smem_launch_ksw_align2(&K, g->n_cu, st));
    HIP_TRY(hipEventRecord(ev[1], st));
    HIP_TRY(hipMemcpyAsync(out, dr.p, sizeof(smem::KswAResult) * n, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, ev[0], ev[1]));
    if (kernel_ms) *kernel_ms = ms;
    return SMEM_OK;
}

void smem_aln_opt_default(smem_aln_opt_t* o) {
    if (!o) return;
    std::memset(o, 0, sizeof(*o));
    smem_ksw_opt_default(&o->sc);
    // mem_opt_init (software/bwamem.c:47-70)
    o->a = 1, o->w = 100, o->zdrop = 100, o->pen_clip5 = o->pen_clip3 = 5, o->min_seed_len = 19;
}

static_assert(sizeof(smem_alnreg_t) == sizeof(smem::AlnReg), "region layout");
static_assert(sizeof(smem_chain_t) == sizeof(smem::OutChain), "chain layout");
static_assert(sizeof(smem_seed_t) == sizeof(smem::SeedRec), "seed layout");

// mem_opt_t scoring / extension fields into the kernel parameters
static void aln_opt_params(const smem_aln_opt_t* opt, smem::AlnParams& P) {
    std::memcpy(P.mat, opt->sc.mat, 25);
    P.o_del = opt->sc.o_del, P.e_del = opt->sc.e_del, P.o_ins = opt->sc.o_ins, P.e_ins = opt->sc.e_ins;
    P.a = opt->a, P.w = opt->w, P.zdrop = opt->zdrop, P.pen_clip5 = opt->pen_clip5, P.pen_clip3 = opt->pen_clip3;
    P.min_seed_len = opt->min_seed_len;
    // ksw_qinit's bias and largest score (software/ksw.c:78-85)
    uint8_t sh = 127, md = 0;
    for (int k = 0; k < 25; ++k) {
        if (opt->sc.mat[k] < (int8_t)sh) sh = (uint8_t)opt->sc.mat[k];
        if (opt->sc.mat[k] > (int8_t)md) md = (uint8_t)opt->sc.mat[k];
    }
    P.top = md, P.sw_shift = (uint8_t)(256 - sh);
}

static int aln_opt_ok(const smem_aln_opt_t* opt) {
    return opt && opt->sc.e_del >= 1 && opt->sc.e_ins >= 1 && opt->sc.o_del >= 0 && opt->sc.o_ins >= 0 && opt->a >= 1 &&
           opt->w >= 0;
}

static int load_pac_impl(smem_gpu_t* g, const uint8_t* pac, int64_t l_pac);
int smem_gpu_load_pac(smem_gpu_t* g, const uint8_t* pac, int64_t l_pac) {
    g_err[0] = 0;
    gpu_wait(g);
    return load_pac_impl(g, pac, l_pac);
}

static int load_pac_impl(smem_gpu_t* g, const uint8_t* pac, int64_t l_pac) {
    if (!g || !pac || l_pac <= 0 || 2 * (uint64_t)l_pac != g->L2[4])
        return fail(SMEM_E_ARG, "smem_gpu_load_pac: pac does not belong to this index (2 l_pac != seq_len)");
    // under the device lock and after every queued kernel: no batch may be
    // reading the old copy, and a failed upload leaves no half-written one
    std::lock_guard<std::mutex> lk(g->mu);
    if (int r = gpu_check(g)) return r;
    HIP_TRY(hipSetDevice(g->device));
    if (g->d_pac) {
        HIP_TRY(hipDeviceSynchronize());
        (void)hipFree(g->d_pac);
        g->d_pac = nullptr;
    }
    g->l_pac = 0;
    const uint64_t bytes = (uint64_t)(l_pac + 3) / 4;
    uint8_t* p = nullptr;
    hipError_t e = hipMalloc(&p, bytes + 64);
    if (e != hipSuccess) return fail(SMEM_E_NOMEM, "smem_gpu_load_pac: hipMalloc", e);
    e = hipMemcpy(p, pac, bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemset(p + bytes, 0, 64);
    if (e != hipSuccess) {
        (void)hipFree(p);
        return fail(SMEM_E_DEVICE, "smem_gpu_load_pac: upload", e);
    }
    g->d_pac = p;
    g->l_pac = l_pac;
    return SMEM_OK;
}

// SMEM_ALN_STREAMS=1: the light and heavy reads' kernels one after the other
// on the batch's stream (default 2: side by side)
static bool aln_two_streams() {
    const char* e = getenv("SMEM_ALN_STREAMS");
    return !(e && atoi(e) == 1);
}
// SMEM_ALN_LIGHT_CLAIMS: beside the heavy kernels, a light wave's claims of 4
// reads before it exits (default 1; 0: persistent)
static uint32_t aln_light_claims() {
    const char* e = getenv("SMEM_ALN_LIGHT_CLAIMS");
    return e ? (uint32_t)std::max(0, atoi(e)) : 1u;
}

// reads with at least this many chains, or seeds, take the heavy path
// (SMEM_ALN_HEAVY_MIN / SMEM_ALN_HEAVY_SEEDS override; a zero chain count =
// never): tandem-repeat reads carry hundreds to thousands of chains or seeds,
// and one wave walking them alone kept the whole launch waiting (0.5 s for
// one read, profiles/r02/aln/)
static uint32_t aln_heavy_min() {
    const char* e = getenv("SMEM_ALN_HEAVY_MIN");
    return e ? (uint32_t)atoi(e) : 17u;
}
// (seeds: 16 since round 4 -- human-like 71.8 -> 70.5 ms per 1M reads,
// uniform 29.0 -> 28.9; 8-48 swept, profiles/r04/aln/heavy_seeds_sweep.txt)
static uint32_t aln_heavy_seeds() {
    const char* e = getenv("SMEM_ALN_HEAVY_SEEDS");
    return e ? (uint32_t)atoi(e) : 16u;
}
// SMEM_ALN_CAND=0: the heavy walk without the candidate index (the bin hash
// of the regions made so far, as before it)
static bool aln_cand_on() {
    const char* e = getenv("SMEM_ALN_CAND");
    return !e || atoi(e) != 0;
}
// the heavy walk's waves per CU (SMEM_ALN_WALK_WAVES; aln_heavy_kernel takes 132 VGPRs: at most
// 12; 4, 8 and 12 measured the same, profiles/r06/aln/s6e_walk_ab.log: the walk's end is its
// longest reads, hence the giant split)
static uint32_t aln_walk_wpc() {
    const char* e = getenv("SMEM_ALN_WALK_WAVES");
    const int v = e ? atoi(e) : smem::ALN_WALK_WAVES;
    return (uint32_t)std::max(4, std::min(16, v / 4 * 4));
}
// the giant split's reads (SMEM_ALN_GIANTS, default 2048; 0: off): the heaviest heavy reads by
// seeds + chains (a read of ~10k seeds walks ~17 ms on its wave; the human-like profile's 1M reads
// hold dozens), their passes and walk on the batch's third stream from the start.  Measured on
// the human-like 1M reads (profiles/r06/aln/s6q_giants.log): 0 63.5 ms, 128 64.8 (giants after
// the others' passes), 512 60.4, 1024 59.7, 2048 59.4, 4096 61.9, all 38k heavy reads 63.2
static uint32_t aln_giants() {
    const char* e = getenv("SMEM_ALN_GIANTS");
    return e ? (uint32_t)std::max(0, atoi(e)) : 2048u;
}
// SMEM_ALN_LANE=0: no regions computed ahead one seed per lane (the walks
// extend every seed one wave per problem, round-2 style)
static bool aln_lane_on() {
    const char* e = getenv("SMEM_ALN_LANE");
    return !(e && atoi(e) == 0);
}

// mem_chain2aln of every chain of every read (P filled, ctr zeroed for
// smem::ALN_CTRS): heavy reads listed, their chains' and seeds' regions
// computed ahead one wave per chain and walked one wave per read; the other
// reads one wave each
// classify -> (heavy reads: chain tasks, then the walk, on st) beside (light
// reads on st2), joined back into st.  The two sets of reads write disjoint
// slots (regions and sort scratch at each read's seed offset, n_regs per read)
// and claim from different counters, so they can share the GPU: the light
// kernel fills the CUs the walk's few long reads leave idle.  st2 == nullptr:
// everything on st.
// after a run_aln with the guarded walk: fail if any walk tripped its guard.
// SMEM_ALN_STATS: print the heavy path's counters (regions the chain tasks
// computed ahead, the walk's regions taken from them / computed serially)
static int aln_guard_check(const smem::AlnParams& P, hipStream_t st, uint64_t* hs) {
    if (getenv("SMEM_ALN_STATS")) {
        uint32_t c[smem::ALN_CTRS], nt = 0;
        HIP_TRY(hipMemcpyAsync(c, P.ctr, sizeof(c), hipMemcpyDeviceToHost, st));
        uint32_t nht = 0;
        if (P.lane_on) HIP_TRY(hipMemcpyAsync(&nt, P.lq + smem::LQ_NTASK, sizeof(nt), hipMemcpyDeviceToHost, st));
        if (P.lane_on) HIP_TRY(hipMemcpyAsync(&nht, P.hlq + smem::LQ_NTASK, sizeof(nht), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        fprintf(stderr, "[smem aln] heavy path: %u reads, %u chains (%u ran mem_chain2aln_short's SW), %u seed regions "
                        "computed ahead, %u used by the walks, %u computed serially in the walks; lane tasks %u "
                        "light + %u heavy (%u left to one wave each)\n", c[2], c[11], c[12], c[8], c[9], c[10], nt,
                nht, c[14]);
    }
    if (!P.walk_guard) return SMEM_OK;
    hs[2] = 0;
    HIP_TRY(hipMemcpyAsync(&hs[2], P.ctr + 15, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (const uint32_t trips = (uint32_t)hs[2]) {
        snprintf(g_err, sizeof(g_err), "chains -> regions: the inlined heavy-read walk tripped its guard %u times", trips);
        return SMEM_E_INTERNAL;
    }
    return SMEM_OK;
}

// hs: >= 4 words of pinned host memory for the scalars copied back (never
// pageable or stack memory: a copy must not outlive the call's frame)
static int run_aln(smem_gpu_t* g, smem::AlnParams& P, uint64_t n_chains, uint64_t n_seeds, bool long_reads,
                   AlnHeavyBufs& H, uint64_t* hs, hipStream_t st, hipStream_t st2 = nullptr,
                   hipEvent_t ev_join = nullptr, hipStream_t st3 = nullptr, hipEvent_t ev_giant = nullptr) {
    const int n = P.n_reads;
    P.heavy_min = aln_heavy_min();
    P.heavy_seeds = aln_heavy_seeds();
    {   // SMEM_ALN_HASH_MIN: chains from which a heavy read's walk hashes its regions (tests force 1)
        const char* e = getenv("SMEM_ALN_HASH_MIN");
        P.hash_min = e ? (uint32_t)std::max(1, atoi(e)) : 64u;
        const char* l = getenv("SMEM_ALN_SPEC_LOCAL");
        P.spec_local = l ? (uint32_t)atoi(l) : 0u;
        // SMEM_ALN_WALK_INLINE=1: the heavy-read walk inlined, every loop
        // iteration counted against a guard (diagnostic of the round-2 hang)
        const char* w = getenv("SMEM_ALN_WALK_INLINE");
        P.walk_guard = (w && atoi(w) > 0) ? (atoi(w) > 1 ? (uint32_t)atoi(w) : (1u << 26)) : 0u;
    }
    P.lane_on = aln_lane_on() && n > 0 ? 1u : 0u;
    if (P.lane_on) {
        const uint64_t nt = std::max<uint64_t>(n_chains, 1), nht = std::max<uint64_t>(n_seeds, 1);
        HIP_TRY(H.pre.grow(std::max<uint64_t>(n_seeds, 1)));
        HIP_TRY(H.pre_ok.grow(std::max<uint64_t>(n_seeds, 1)));
        HIP_TRY(H.span.grow(2 * std::max<uint64_t>(n_chains, 1)));
        HIP_TRY(H.sdec.grow(std::max<uint64_t>(n_chains, 1)));
        HIP_TRY(H.tasks.grow(nt));
        HIP_TRY(H.torder.grow(nt));
        HIP_TRY(H.tfail.grow(nt));
        HIP_TRY(H.lq.grow(smem::LQ_WORDS));
        HIP_TRY(H.htasks.grow(nht));
        HIP_TRY(H.htorder.grow(nht));
        HIP_TRY(H.htfail.grow(nht));
        HIP_TRY(H.hlq.grow(smem::LQ_WORDS));
        HIP_TRY(hipMemsetAsync(H.hlq.p, 0, sizeof(uint32_t) * smem::LQ_WORDS, st));
        HIP_TRY(H.chain_read.grow(std::max<uint64_t>(n_chains, 1)));
        HIP_TRY(H.swlist.grow(std::max<uint64_t>(n_chains, 1)));
        HIP_TRY(H.short_ok.grow(std::max<uint64_t>(n_chains, 1)));
        HIP_TRY(H.pre_short.grow(std::max<uint64_t>(n_chains, 1)));
        HIP_TRY(hipMemsetAsync(H.lq.p, 0, sizeof(uint32_t) * smem::LQ_WORDS, st));
        P.pre = H.pre.p, P.pre_ok = H.pre_ok.p, P.span = H.span.p, P.sdec = H.sdec.p;
        P.tasks = H.tasks.p, P.torder = H.torder.p, P.tfail = H.tfail.p, P.lq = H.lq.p;
        P.chain_read = H.chain_read.p, P.swlist = H.swlist.p, P.short_ok = H.short_ok.p, P.pre_short = H.pre_short.p;
        P.htasks = H.htasks.p, P.hlq = H.hlq.p;
    }
    uint32_t n_heavy = 0;
    if (P.heavy_min && n > 0) {
        HIP_TRY(H.heavy.grow(n));
        HIP_TRY(H.hcnt.grow(n));
        HIP_TRY(H.hscnt.grow(n));
        P.heavy = H.heavy.p, P.hcnt = H.hcnt.p, P.hscnt = H.hscnt.p;
        HIP_TRY(smem_launch_aln_classify(&P, st));
        hs[0] = 0;
        HIP_TRY(hipMemcpyAsync(&hs[0], P.ctr + 2, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        n_heavy = (uint32_t)hs[0];
    }
    P.walk_wpc = aln_walk_wpc();
    P.walk_waves = 0;
    P.rgiant = nullptr, P.gtasks = nullptr, P.glq = nullptr;
    // the giant split: heavy[] reordered (most seeds + chains first), its first n_giant reads the
    // giants (lane path, candidate index, three streams)
    const uint32_t n_giant = (P.lane_on && n_heavy && st2 && st3 && ev_join && ev_giant && aln_cand_on())
                                 ? std::min<uint32_t>(n_heavy, aln_giants()) : 0u;
    if (n_giant) {
        const uint64_t nht = std::max<uint64_t>(n_seeds, 1);
        HIP_TRY(H.heavy2.grow(n_heavy));
        HIP_TRY(H.hcnt2.grow(n_heavy));
        HIP_TRY(H.hscnt2.grow(n_heavy));
        HIP_TRY(H.rgiant.grow(n));
        HIP_TRY(H.gctr.grow(smem::ALN_CTRS));
        HIP_TRY(H.gtasks.grow(nht));
        HIP_TRY(H.gtorder.grow(nht));
        HIP_TRY(H.gtfail.grow(nht));
        HIP_TRY(H.glq.grow(smem::LQ_WORDS));
        HIP_TRY(hipMemsetAsync(H.gctr.p, 0, sizeof(uint32_t) * smem::ALN_CTRS, st));
        HIP_TRY(hipMemsetAsync(H.glq.p, 0, sizeof(uint32_t) * smem::LQ_WORDS, st));
        HIP_TRY(smem_launch_aln_heavy_split(&P, n_heavy, n_giant, H.heavy2.p, H.hcnt2.p, H.hscnt2.p, H.rgiant.p,
                                            H.gctr.p, P.ctr, st));
        P.heavy = H.heavy2.p, P.hcnt = H.hcnt2.p, P.hscnt = H.hscnt2.p;
        P.rgiant = H.rgiant.p, P.gtasks = H.gtasks.p, P.glq = H.glq.p;
    }
    smem::CandParams C{}, Cg{};
    uint64_t m_giant = 0;  // the giants' candidate slots (first in the index arrays)
    if (n_heavy && P.lane_on) {  // the walk's scratch (its chains were prepared by the lane path)
        // the bin hash (0.54 GB at 256 CUs) only serves a walk without the candidate index
        // (aln_heavy_kernel: `hashed` needs !indexed)
        if (!aln_cand_on()) HIP_TRY(H.ht.grow((size_t)g->n_cu * P.walk_wpc * smem::ALN_HT));
        HIP_TRY(H.rnext.grow(std::max<uint64_t>(n_seeds, 1)));
        P.ht = H.ht.p, P.rnext = H.rnext.p;
        if (aln_cand_on()) {
            // the candidate index's size: every heavy read's seeds and chains, in two
            // instances under the giant split -- the giants (heavy[0 .. n_giant)) and the
            // rest (heavy[n_giant ..)), each with its read -> segment map (hord, the other
            // instance's reads unmapped) and its slots (the giants' first)
            const uint32_t nr = n_heavy - n_giant;
            smem::AlnParams Pr = P;
            Pr.heavy = P.heavy + n_giant, Pr.hcnt = P.hcnt + n_giant, Pr.hscnt = P.hscnt + n_giant;
            HIP_TRY(H.ccnt.grow(std::max<uint32_t>(nr, 1)));
            HIP_TRY(H.coff.grow(nr + 1));
            HIP_TRY(H.chord.grow(std::max(n, 1)));
            HIP_TRY(hipMemsetAsync(H.chord.p, 0xFF, sizeof(uint32_t) * (size_t)std::max(n, 1), st));
            size_t tb = 0;
            HIP_TRY(smem_launch_offsets(nullptr, nullptr, (int)n_heavy, nullptr, &tb, st));
            HIP_TRY(H.tmp.grow(tb + 256));
            if (nr) {
                HIP_TRY(smem_launch_aln_cand_count(&Pr, nr, H.ccnt.p, H.chord.p, st));
                tb = H.tmp.n;
                HIP_TRY(smem_launch_offsets(H.ccnt.p, H.coff.p, (int)nr, H.tmp.p, &tb, st));
            } else {
                HIP_TRY(hipMemsetAsync(H.coff.p, 0, sizeof(uint64_t), st));
            }
            HIP_TRY(hipMemcpyAsync(&hs[1], H.coff.p + nr, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
            hs[3] = 0;
            if (n_giant) {
                HIP_TRY(H.ccnt_g.grow(n_giant));
                HIP_TRY(H.coff_g.grow(n_giant + 1));
                HIP_TRY(H.chord_g.grow(std::max(n, 1)));
                HIP_TRY(hipMemsetAsync(H.chord_g.p, 0xFF, sizeof(uint32_t) * (size_t)std::max(n, 1), st));
                HIP_TRY(smem_launch_aln_cand_count(&P, n_giant, H.ccnt_g.p, H.chord_g.p, st));
                tb = H.tmp.n;
                HIP_TRY(smem_launch_offsets(H.ccnt_g.p, H.coff_g.p, (int)n_giant, H.tmp.p, &tb, st));
                HIP_TRY(hipMemcpyAsync(&hs[3], H.coff_g.p + n_giant, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
            }
            HIP_TRY(hipStreamSynchronize(st));
            const uint64_t m = hs[1];
            m_giant = hs[3];
            const uint64_t mm = std::max<uint64_t>(m + m_giant, 1);
            HIP_TRY(H.ckey.grow(mm));
            HIP_TRY(H.ckey2.grow(mm));
            HIP_TRY(H.cval.grow(mm));
            HIP_TRY(H.cval2.grow(mm));
            HIP_TRY(H.chmax.grow(n_heavy));
            HIP_TRY(H.crb.grow(mm));
            HIP_TRY(H.cre.grow(mm));
            HIP_TRY(H.cq.grow(mm));
            HIP_TRY(H.cmade.grow(mm));
            HIP_TRY(H.cpos_s.grow(std::max<uint64_t>(n_seeds, 1)));
            HIP_TRY(H.cpos_c.grow(std::max<uint64_t>(n_chains, 1)));
            HIP_TRY(H.crng.grow(std::max<uint64_t>(n_seeds, 1)));
            const uint64_t mg = m_giant;
            C.key = H.ckey.p + mg, C.key2 = H.ckey2.p + mg, C.val = H.cval.p + mg, C.val2 = H.cval2.p + mg;
            C.off = H.coff.p, C.hmax = H.chmax.p + n_giant, C.hord = H.chord.p, C.n_heavy = nr, C.m = m;
            C.n_chains = n_chains;
            size_t sb = 0;
            HIP_TRY(smem_launch_aln_cand(&Pr, &C, nullptr, &sb, g->n_cu, st));
            HIP_TRY(H.ctmp.grow(sb + 256));
            if (n_giant) {
                Cg.key = H.ckey.p, Cg.key2 = H.ckey2.p, Cg.val = H.cval.p, Cg.val2 = H.cval2.p, Cg.off = H.coff_g.p;
                Cg.hmax = H.chmax.p, Cg.hord = H.chord_g.p, Cg.n_heavy = n_giant, Cg.m = mg, Cg.n_chains = n_chains;
                sb = 0;
                HIP_TRY(smem_launch_aln_cand(&P, &Cg, nullptr, &sb, g->n_cu, st));
                HIP_TRY(H.ctmp_g.grow(sb + 256));
            }
            P.cand_rb = H.crb.p, P.cand_re = H.cre.p, P.cand_q = H.cq.p, P.cand_made = H.cmade.p;
            P.cand_pos_s = H.cpos_s.p, P.cand_pos_c = H.cpos_c.p, P.cand_rng = H.crng.p;
        }
    } else if (n_heavy) {
        HIP_TRY(H.hoff.grow(n_heavy + 1));
        size_t tb = 0;
        HIP_TRY(smem_launch_offsets(nullptr, nullptr, (int)n_heavy, nullptr, &tb, st));
        HIP_TRY(H.tmp.grow(tb + 256));
        tb = H.tmp.n;
        HIP_TRY(smem_launch_offsets(H.hcnt.p, H.hoff.p, (int)n_heavy, H.tmp.p, &tb, st));
        HIP_TRY(H.pre.grow(std::max<uint64_t>(n_seeds, 1)));
        if (P.spec_local) HIP_TRY(H.loc.grow(std::max<uint64_t>(n_seeds, 1)));  // only SMEM_ALN_SPEC_LOCAL reads it
        HIP_TRY(H.pre_ok.grow(std::max<uint64_t>(n_seeds, 1)));
        HIP_TRY(H.pre_short.grow(std::max<uint64_t>(n_chains, 1)));
        HIP_TRY(H.short_ok.grow(std::max<uint64_t>(n_chains, 1)));
        HIP_TRY(H.span.grow(2 * std::max<uint64_t>(n_chains, 1)));
        HIP_TRY(H.ht.grow((size_t)g->n_cu * P.walk_wpc * smem::ALN_HT));
        HIP_TRY(H.rnext.grow(std::max<uint64_t>(n_seeds, 1)));
        P.hoff = H.hoff.p, P.pre = H.pre.p, P.loc = H.loc.p, P.pre_ok = H.pre_ok.p, P.pre_short = H.pre_short.p;
        P.short_ok = H.short_ok.p, P.span = H.span.p, P.ht = H.ht.p, P.rnext = H.rnext.p;
    }
    if (P.lane_on) {
        // every chain prepared and its tasks listed; then the heavy reads'
        // tasks' passes and their walk (the critical path: one wave walks a
        // read's thousands of chains) on st, beside the light reads' passes and
        // walk on st2
        const int lr = long_reads ? 1 : 0;
        // the heavy chains' short SW (prep part 2) is enqueued after the light reads' stream
        // has forked off: their passes need only the task lists (part 1)
        HIP_TRY(smem_launch_aln_prep(&P, n_chains, g->n_cu, (n_heavy && st2 && ev_join) ? 1 : 3, st));
        smem::AlnParams Ph = P;  // the heavy list (under the giant split: the rest)
        Ph.tasks = H.htasks.p, Ph.torder = H.htorder.p, Ph.tfail = H.htfail.p, Ph.lq = H.hlq.p;
        Ph.heavy = P.heavy + n_giant, Ph.hcnt = P.hcnt + n_giant, Ph.hscnt = P.hscnt + n_giant;
        if (Ph.cand_made) {
            Ph.cand_rb += m_giant, Ph.cand_re += m_giant, Ph.cand_q += m_giant, Ph.cand_made += m_giant;
        }
        // the heavy walk's candidate index once the regions it holds are computed
        auto cand = [&]() -> hipError_t {
            if (!Ph.cand_made) return hipSuccess;
            size_t sb = H.ctmp.n;
            return smem_launch_aln_cand(&Ph, &C, H.ctmp.p, &sb, g->n_cu, st);
        };
        if (n_giant) {
            // four queues of work, each enqueued before the host blocks again (the candidate
            // index's segmented sort reads its partition sizes back):
            //   st:  the rest's passes, then their candidate index and walk
            //   st2: the light reads' passes and walk
            //   st3: the giants' passes, candidate index and walk (one wave each)
            smem::AlnParams Pg = P;
            Pg.tasks = H.gtasks.p, Pg.torder = H.gtorder.p, Pg.tfail = H.gtfail.p, Pg.lq = H.glq.p;
            Pg.ctr = H.gctr.p, Pg.walk_waves = n_giant;
            // SMEM_ALN_GIANT_FIRST (default 2): the giants' passes and candidate index run
            // before the other heavy reads' passes start (ev_giant, recorded twice: the
            // waits enqueued between take the first record), the light reads' passes
            // beside them from the start (1: the light reads' wait too; 0: nobody waits)
            // -- the lane passes hold every CU until their queues drain, so the giants'
            // small kernels beside them waited ~30 ms for CUs (profiles/r06/aln, the s6n
            // timeline); their walk, one wave a read, then runs beside the rest
            const char* gf = getenv("SMEM_ALN_GIANT_FIRST");
            const int first = gf ? atoi(gf) : 2;
            HIP_TRY(hipEventRecord(ev_join, st));  // the task lists are made
            if (first != 1) HIP_TRY(hipStreamWaitEvent(st2, ev_join, 0));
            HIP_TRY(smem_launch_aln_prep(&P, n_chains, g->n_cu, 2, st));  // the heavy chains' short SW
            HIP_TRY(hipEventRecord(ev_giant, st));
            HIP_TRY(hipStreamWaitEvent(st3, ev_giant, 0));
            HIP_TRY(smem_launch_aln_passes(&Pg, g->n_cu, lr, st3));
            {
                size_t sb = H.ctmp_g.n;
                HIP_TRY(smem_launch_aln_cand(&Pg, &Cg, H.ctmp_g.p, &sb, g->n_cu, st3));
            }
            if (first) {
                HIP_TRY(hipEventRecord(ev_giant, st3));
                HIP_TRY(hipStreamWaitEvent(st, ev_giant, 0));
                if (first == 1) HIP_TRY(hipStreamWaitEvent(st2, ev_giant, 0));
            }
            HIP_TRY(smem_launch_aln_heavy(&Pg, g->n_cu, lr, 2, st3));
            HIP_TRY(hipEventRecord(ev_giant, st3));
            HIP_TRY(smem_launch_aln_passes(&Ph, g->n_cu, lr, st));
            HIP_TRY(smem_launch_aln_passes(&P, g->n_cu, lr, st2));
            P.light_claims = aln_light_claims();
            HIP_TRY(smem_launch_aln(&P, g->n_cu, lr, st2));
            P.light_claims = 0;
            HIP_TRY(hipEventRecord(ev_join, st2));
            if (n_heavy > n_giant) {
                HIP_TRY(cand());
                HIP_TRY(smem_launch_aln_heavy(&Ph, g->n_cu, lr, 2, st));
            }
            HIP_TRY(hipStreamWaitEvent(st, ev_join, 0));
            HIP_TRY(hipStreamWaitEvent(st, ev_giant, 0));
            return SMEM_OK;
        }
        if (n_heavy && st2 && ev_join) {
            HIP_TRY(hipEventRecord(ev_join, st));
            HIP_TRY(hipStreamWaitEvent(st2, ev_join, 0));
            HIP_TRY(smem_launch_aln_prep(&P, n_chains, g->n_cu, 2, st));  // the heavy chains' short SW
            HIP_TRY(smem_launch_aln_passes(&Ph, g->n_cu, lr, st));
            HIP_TRY(cand());
            HIP_TRY(smem_launch_aln_heavy(&Ph, g->n_cu, lr, 2, st));
            HIP_TRY(smem_launch_aln_passes(&P, g->n_cu, lr, st2));
            P.light_claims = aln_light_claims();
            HIP_TRY(smem_launch_aln(&P, g->n_cu, lr, st2));
            P.light_claims = 0;
            HIP_TRY(hipEventRecord(ev_join, st2));
            HIP_TRY(hipStreamWaitEvent(st, ev_join, 0));
            return SMEM_OK;
        }
        if (n_heavy) {
            HIP_TRY(smem_launch_aln_passes(&Ph, g->n_cu, lr, st));
            HIP_TRY(cand());
            HIP_TRY(smem_launch_aln_heavy(&Ph, g->n_cu, lr, 2, st));
        }
        HIP_TRY(smem_launch_aln_passes(&P, g->n_cu, lr, st));
        HIP_TRY(smem_launch_aln(&P, g->n_cu, lr, st));
        return SMEM_OK;
    }
    if (n_heavy) {
        if (st2 && ev_join) {
            // the heavy kernels first (their chain tasks then the walk are the
            // critical path); classify finished (synchronised above), so st2
            // has nothing to wait for
            HIP_TRY(smem_launch_aln_heavy(&P, g->n_cu, long_reads ? 1 : 0, 3, st));
            P.light_claims = aln_light_claims();  // its blocks retire, so the walk finds CU slots
            HIP_TRY(smem_launch_aln(&P, g->n_cu, long_reads ? 1 : 0, st2));
            P.light_claims = 0;
            HIP_TRY(hipEventRecord(ev_join, st2));
            HIP_TRY(hipStreamWaitEvent(st, ev_join, 0));
            return SMEM_OK;
        }
        HIP_TRY(smem_launch_aln_heavy(&P, g->n_cu, long_reads ? 1 : 0, 3, st));
    }
    HIP_TRY(smem_launch_aln(&P, g->n_cu, long_reads ? 1 : 0, st));
    return SMEM_OK;
}

int smem_batch_chain2aln(smem_batch_t* b, const smem_aln_opt_t* opt) {
    g_err[0] = 0;
    if (!b || !b->chain_ran || !b->chain_filtered)
        return fail(SMEM_E_ARG, "smem_batch_chain2aln: run smem_batch_chain with filter = 1 first");
    if (!aln_opt_ok(opt)) return fail(SMEM_E_ARG, "smem_batch_chain2aln: scoring needs e >= 1, o >= 0, a >= 1, w >= 0");
    smem_gpu_t* g = b->g;
    if (!g->d_pac) return fail(SMEM_E_ARG, "smem_batch_chain2aln: no .pac loaded (smem_gpu_load_pac)");
    if (b->max_len > 1024) return fail(SMEM_E_ARG, "smem_batch_chain2aln: reads longer than 1024 bp");
    BatchCall call(b, aln_two_streams());
    if (call.rc) return call.rc;
    b->aln_ran = b->aln_fetched = false;
    const int n = b->n_reads;
    const uint64_t ns = std::max<uint64_t>(b->tot_seeds, 1);
    HIP_TRY(b->d_aln_srt.grow(ns + 1));
    HIP_TRY(b->d_aln_raw.grow(ns + 1));
    HIP_TRY(b->d_aln_nregs.grow(std::max(n, 1)));
    HIP_TRY(b->d_aln_regoff.grow(n + 1));
    HIP_TRY(b->d_aln_ctr.grow(smem::ALN_CTRS));
    size_t tmp = 0;
    HIP_TRY(smem_launch_offsets(nullptr, nullptr, std::max(n, 1), nullptr, &tmp, b->st));
    HIP_TRY(b->d_sa_tmp.grow(tmp + 256));
    smem::AlnParams P;
    std::memset(&P, 0, sizeof(P));
    P.codes = b->d_codes.p, P.offs = b->d_offs.p, P.chains = b->d_out_chain.p, P.chain_off = b->d_chain_off.p;
    P.seeds = b->d_out_seed.p;
    P.seed_off = b->d_seed_off.p;  // a read's chains' seeds are contiguous: its region capacity
    P.pac = g->d_pac, P.l_pac = g->l_pac, P.n_reads = n;
    P.max_len = b->read_len_max > 0 ? b->read_len_max : b->max_len;
    aln_opt_params(opt, P);
    P.srt = b->d_aln_srt.p, P.raw = b->d_aln_raw.p, P.n_regs = b->d_aln_nregs.p, P.ctr = b->d_aln_ctr.p;
    // diagnostics: SMEM_ALN_CYCLES=<file> writes the shader cycles each read took (u64 per read),
    // and <file>.walk the heavy walk's split (4 x u64 per read: cycles in chain_full, cycles in the
    // bin-hash containment walks, chains over 64 seeds | their seeds << 32, bin-list hops)
    const char* cyc_path = getenv("SMEM_ALN_CYCLES");
    DevBuf<uint64_t> d_cyc;
    struct Free {
        DevBuf<uint64_t>& b;
        ~Free() { b.release(); }  // every return path, HIP_TRY's included
    } free_cyc{d_cyc};
    if (cyc_path) {
        HIP_TRY(d_cyc.ensure(5 * (uint64_t)std::max(n, 1)));
        HIP_TRY(hipMemsetAsync(d_cyc.p, 0, 5 * sizeof(uint64_t) * (uint64_t)std::max(n, 1), b->st));
        P.cyc = d_cyc.p;
    }
    // SMEM_ALN_SPLIT=1: aln_kernel's cycles by phase and its counts (smem::Split), on stderr
    const bool split = getenv("SMEM_ALN_SPLIT") && atoi(getenv("SMEM_ALN_SPLIT"));
    DevBuf<uint64_t> d_split;
    Free free_split{d_split};
    if (split) {
        HIP_TRY(d_split.ensure(smem::ALN_SPLITS));
        HIP_TRY(hipMemsetAsync(d_split.p, 0, smem::ALN_SPLITS * sizeof(uint64_t), b->st));
        P.split = d_split.p;
    }
    HIP_TRY(hipMemsetAsync(b->d_aln_ctr.p, 0, smem::ALN_CTRS * sizeof(uint32_t), b->st));
    HIP_TRY(hipEventRecord(b->ev[0], b->st));
    // the light reads' kernels on the pair's low-priority stream
    if (aln_two_streams() && !b->ev_join) HIP_TRY(hipEventCreateWithFlags(&b->ev_join, hipEventDisableTiming));
    if (aln_two_streams() && !b->ev_giant) HIP_TRY(hipEventCreateWithFlags(&b->ev_giant, hipEventDisableTiming));
    if (int rc = run_aln(g, P, b->tot_chains, b->tot_seeds, b->max_len > 256, b->aln_heavy, b->h_tot.p + 8, b->st,
                         aln_two_streams() ? b->st2 : nullptr, b->ev_join, aln_two_streams() ? b->st3 : nullptr,
                         b->ev_giant))
        return rc;
    if (int rc = aln_guard_check(P, b->st, b->h_tot.p + 8)) return rc;
    tmp = b->d_sa_tmp.n;
    HIP_TRY(smem_launch_offsets(b->d_aln_nregs.p, b->d_aln_regoff.p, n, b->d_sa_tmp.p, &tmp, b->st));
    HIP_TRY(hipMemcpyAsync(b->h_tot.p + 5, b->d_aln_regoff.p + n, sizeof(uint64_t), hipMemcpyDeviceToHost, b->st));
    HIP_TRY(hipStreamSynchronize(b->st));
    b->tot_regs = n > 0 ? b->h_tot.p[5] : 0;
    if (b->tot_regs > b->tot_seeds) return fail(SMEM_E_INTERNAL, "smem_batch_chain2aln: more regions than seeds");
    HIP_TRY(b->d_aln_out.grow(std::max<uint64_t>(b->tot_regs, 1)));
    P.reg_off = b->d_aln_regoff.p, P.out = b->d_aln_out.p;
    HIP_TRY(smem_launch_aln_write(&P, b->st));
    HIP_TRY(hipEventRecord(b->ev[1], b->st));
    INJECT(ST_ALN);
    HIP_TRY(hipStreamSynchronize(b->st));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, b->ev[0], b->ev[1]));
    b->stats.aln_ms = ms;
    b->stats.n_regs = b->tot_regs;
    if (cyc_path && n > 0) {
        std::vector<uint64_t> h(5 * (uint64_t)n);
        HIP_TRY(hipMemcpy(h.data(), d_cyc.p, sizeof(uint64_t) * h.size(), hipMemcpyDeviceToHost));
        if (FILE* f = fopen(cyc_path, "wb")) {
            fwrite(h.data(), sizeof(uint64_t), n, f);
            fclose(f);
        }
        if (FILE* f = fopen((std::string(cyc_path) + ".walk").c_str(), "wb")) {
            fwrite(h.data() + n, sizeof(uint64_t), 4 * (uint64_t)n, f);
            fclose(f);
        }
    }
    if (split) {
        uint64_t h[smem::ALN_SPLITS];
        HIP_TRY(hipMemcpy(h, d_split.p, sizeof(h), hipMemcpyDeviceToHost));
        fprintf(stderr, "aln split:");
        for (int k = 0; k < smem::ALN_SPLITS; ++k) fprintf(stderr, " %llu", (unsigned long long)h[k]);
        fprintf(stderr, "\n");
    }
    b->aln_ran = true;
    b->aln_fetched = false;
    return SMEM_OK;
}

int smem_batch_aln_results(const smem_batch_t* b, const smem_alnreg_t** regs, const uint64_t** reg_off,
                           uint64_t* n_regs) {
    if (!b || !b->aln_fetched) return SMEM_E_ARG;
    if (regs) *regs = reinterpret_cast<const smem_alnreg_t*>(b->h_aln_regs.p);
    if (reg_off) *reg_off = b->h_aln_regoff.p;
    if (n_regs) *n_regs = b->tot_regs;
    return SMEM_OK;
}

int smem_chain2aln(smem_gpu_t* g, int n_reads, const uint8_t* codes, const uint64_t* offs, const smem_chain_t* chains,
                   const uint64_t* chain_off, const smem_seed_t* seeds, uint64_t n_seeds, const uint8_t* pac,
                   int64_t l_pac, const smem_aln_opt_t* opt, smem_alnreg_t* regs, uint64_t* reg_off,
                   double* kernel_ms) {
    g_err[0] = 0;
    if (!g || n_reads < 0 || !opt || !reg_off || (n_reads > 0 && (!codes || !offs || !chain_off)) || l_pac <= 0)
        return fail(SMEM_E_ARG, "smem_chain2aln: bad arguments");
    if (!pac && !(g->d_pac && g->l_pac == l_pac))
        return fail(SMEM_E_ARG, "smem_chain2aln: no pac given and none resident for this l_pac (smem_gpu_load_pac)");
    if (!aln_opt_ok(opt)) return fail(SMEM_E_ARG, "smem_chain2aln: scoring needs e >= 1, o >= 0, a >= 1, w >= 0");
    if (kernel_ms) *kernel_ms = 0.0;
    reg_off[0] = 0;
    if (n_reads == 0) return SMEM_OK;
    // per-read region capacity = its chains' seeds; the host checks every
    // shape the kernel indexes with before anything is launched
    const uint64_t n_chains = chain_off[n_reads];
    std::vector<uint64_t> cap(n_reads + 1, 0);
    bool long_reads = false;
    int max_len = 0;
    for (int r = 0; r < n_reads; ++r) {
        max_len = std::max<int>(max_len, (int)std::min<uint64_t>(offs[r + 1] - offs[r], 1u << 30));
        if (offs[r + 1] < offs[r] || offs[r + 1] - offs[r] > 1024 || chain_off[r + 1] < chain_off[r])
            return fail(SMEM_E_ARG, "smem_chain2aln: read longer than 1024 bp or offsets not ascending");
        long_reads |= offs[r + 1] - offs[r] > 256;
        uint64_t c = 0;
        for (uint64_t k = chain_off[r]; k < chain_off[r + 1]; ++k) {
            const smem_chain_t& ch = chains[k];
            if (ch.n < 0 || ch.seed_off + (uint64_t)ch.n > n_seeds)
                return fail(SMEM_E_ARG, "smem_chain2aln: chain seeds outside seeds[]");
            for (int i = 0; i < ch.n; ++i) {
                const smem_seed_t& s = seeds[ch.seed_off + i];
                if (s.qbeg < 0 || s.len <= 0 || (uint64_t)s.qbeg + s.len > offs[r + 1] - offs[r] || s.rbeg < 0 ||
                    s.rbeg + s.len > 2 * l_pac)
                    return fail(SMEM_E_ARG, "smem_chain2aln: seed outside its read or the text");
            }
            c += (uint64_t)ch.n;
        }
        cap[r + 1] = cap[r] + c;
    }
    const uint64_t n_bases = offs[n_reads], n_cap = cap[n_reads];
    if (n_cap > 0 && !regs) return fail(SMEM_E_ARG, "smem_chain2aln: no region buffer");
    // query codes index the 25-entry scoring matrix: 0..4 only
    for (uint64_t k = offs[0]; k < n_bases; ++k)
        if (codes[k] > 4) return fail(SMEM_E_ARG, "smem_chain2aln: query code > 4");
    {   // each chain's seed range is its sort scratch: ranges must not overlap
        std::vector<std::pair<uint64_t, uint64_t>> rng;
        rng.reserve(n_chains);
        for (uint64_t k = 0; k < n_chains; ++k)
            if (chains[k].n > 0) rng.emplace_back(chains[k].seed_off, chains[k].seed_off + (uint64_t)chains[k].n);
        std::sort(rng.begin(), rng.end());
        for (size_t k = 1; k < rng.size(); ++k)
            if (rng[k].first < rng[k - 1].second) return fail(SMEM_E_ARG, "smem_chain2aln: chains share seeds");
    }
    DevBuf<uint8_t> dcodes, dpac;
    DevBuf<uint64_t> doffs, dchoff, dseedoff, dsrt, dnregs, dregoff;
    DevBuf<smem::OutChain> dch;
    DevBuf<smem::SeedRec> dseeds;
    DevBuf<smem::AlnReg> draw, dout;
    DevBuf<uint32_t> dctr;
    AlnHeavyBufs heavy;
    HostBuf<uint64_t> hs, hnr;  // pinned: the scalars and region counts copied back
    hipEvent_t ev[2] = {nullptr, nullptr};
    struct Guard {
        std::vector<std::function<void()>> f;
        ~Guard() {
            for (auto& x : f) x();
        }
    } guard;
    guard.f.push_back([&] {
        dcodes.release(); dpac.release(); doffs.release(); dchoff.release(); dseedoff.release(); dsrt.release();
        dnregs.release(); dregoff.release(); dch.release(); dseeds.release(); draw.release(); dout.release();
        dctr.release();
        heavy.release();
        hs.release(); hnr.release();
        if (ev[0]) (void)hipEventDestroy(ev[0]);
        if (ev[1]) (void)hipEventDestroy(ev[1]);
    });
    DeviceCall call(g);  // (declared after the buffers: drained before they are freed)
    if (call.rc) return call.rc;
    const hipStream_t st = call.st;
    HIP_TRY(hs.ensure(8));
    HIP_TRY(hnr.ensure((size_t)n_reads));
    HIP_TRY(hipEventCreate(&ev[0]));
    HIP_TRY(hipEventCreate(&ev[1]));
    const uint64_t pac_bytes = (uint64_t)(l_pac + 3) / 4;
    HIP_TRY(dcodes.ensure(n_bases + 64));
    if (pac) HIP_TRY(dpac.ensure(pac_bytes + 64));
    HIP_TRY(doffs.ensure(n_reads + 1));
    HIP_TRY(dchoff.ensure(n_reads + 1));
    HIP_TRY(dseedoff.ensure(n_reads + 1));
    HIP_TRY(dsrt.ensure(n_seeds + 1));
    HIP_TRY(dnregs.ensure(n_reads));
    HIP_TRY(dregoff.ensure(n_reads + 1));
    HIP_TRY(dch.ensure(n_chains + 1));
    HIP_TRY(dseeds.ensure(n_seeds + 1));
    HIP_TRY(draw.ensure(n_cap + 1));
    HIP_TRY(dout.ensure(n_cap + 1));
    HIP_TRY(dctr.ensure(smem::ALN_CTRS));
    if (n_bases) HIP_TRY(hipMemcpyAsync(dcodes.p, codes, n_bases, hipMemcpyHostToDevice, st));
    if (pac) HIP_TRY(hipMemcpyAsync(dpac.p, pac, pac_bytes, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(doffs.p, offs, 8 * (n_reads + 1), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(dchoff.p, chain_off, 8 * (n_reads + 1), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(dseedoff.p, cap.data(), 8 * (n_reads + 1), hipMemcpyHostToDevice, st));
    if (n_chains) HIP_TRY(hipMemcpyAsync(dch.p, chains, sizeof(smem::OutChain) * n_chains, hipMemcpyHostToDevice, st));
    if (n_seeds) HIP_TRY(hipMemcpyAsync(dseeds.p, seeds, sizeof(smem::SeedRec) * n_seeds, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemsetAsync(dctr.p, 0, smem::ALN_CTRS * sizeof(uint32_t), st));
    smem::AlnParams P;
    std::memset(&P, 0, sizeof(P));
    P.codes = dcodes.p, P.offs = doffs.p, P.chains = dch.p, P.chain_off = dchoff.p, P.seeds = dseeds.p;
    P.seed_off = dseedoff.p, P.pac = pac ? dpac.p : g->d_pac, P.l_pac = l_pac, P.n_reads = n_reads;
    P.max_len = max_len;
    aln_opt_params(opt, P);
    P.srt = dsrt.p, P.raw = draw.p, P.n_regs = dnregs.p, P.ctr = dctr.p;
    HIP_TRY(hipEventRecord(ev[0], st));
    if (int rc = run_aln(g, P, n_chains, n_seeds, long_reads, heavy, hs.p, st)) return rc;
    if (int rc = aln_guard_check(P, st, hs.p)) return rc;
    HIP_TRY(hipEventRecord(ev[1], st));
    const uint64_t* nr = hnr.p;
    HIP_TRY(hipMemcpyAsync(hnr.p, dnregs.p, 8 * n_reads, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    for (int r = 0; r < n_reads; ++r) {
        if (nr[r] > cap[r + 1] - cap[r]) return fail(SMEM_E_INTERNAL, "smem_chain2aln: region count past capacity");
        reg_off[r + 1] = reg_off[r] + nr[r];
    }
    const uint64_t n_out = reg_off[n_reads];
    if (n_out) {
        HIP_TRY(hipMemcpyAsync(dregoff.p, reg_off, 8 * (n_reads + 1), hipMemcpyHostToDevice, st));
        P.reg_off = dregoff.p, P.out = dout.p;
        HIP_TRY(smem_launch_aln_write(&P, st));
        HIP_TRY(hipMemcpyAsync(regs, dout.p, sizeof(smem::AlnReg) * n_out, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, ev[0], ev[1]));
    if (kernel_ms) *kernel_ms = ms;
    return SMEM_OK;
}

int smem_batch_stats(const smem_batch_t* b, smem_batch_stats_t* st) {
    if (!b || !st) return SMEM_E_ARG;
    *st = b->stats;
    return SMEM_OK;
}

// ---- streaming: bwa mem's chunk loop (software/fastmap.c:213-228) with its
// kt_for_batch workers (software/kthread_batch.c:29-59) over one device.
// Each worker owns a batch (pinned staging, HIP stream, device buffers) and
// runs whole chunks: stage + H2D, seed + compact, D2H into pinned memory,
// then the caller's callback.  The workers' chunks interleave on the device,
// so one chunk's copies overlap another's kernels.
int smem_gpu_seed_stream(smem_gpu_t* g, int64_t n_reads, const uint8_t* codes, const uint64_t* offs,
                         const smem_opt_t* opt, int chunk_reads, int n_workers, int flags, smem_chunk_fn fn, void* ctx,
                         smem_stream_stats_t* stats) {
    g_err[0] = 0;
    if (!g || !opt || n_reads < 0 || (n_reads > 0 && (!codes || !offs)) || chunk_reads <= 0 || n_workers <= 0 ||
        n_workers > 64 || (flags & ~(SMEM_STREAM_PAIRS | SMEM_STREAM_PACKED | SMEM_STREAM_RELEASE)))
        return fail(SMEM_E_ARG, "smem_gpu_seed_stream: bad arguments");
    const bool pairs = flags & SMEM_STREAM_PAIRS, packed = flags & SMEM_STREAM_PACKED;
    if (pairs) {
        if (n_reads & 1) return fail(SMEM_E_ARG, "smem_gpu_seed_stream: pairs need an even read count");
        chunk_reads = std::max(2, chunk_reads & ~1);  // both mates of a pair in one chunk (software/bwamem.c:1600-1609)
    }
    const int64_t n_chunks = (n_reads + chunk_reads - 1) / chunk_reads;
    // the largest chunk: reads, bases, read length
    int max_len = 1;
    uint64_t max_bases = 1;
    for (int64_t c = 0; c < n_chunks; ++c) {
        const int64_t a = c * chunk_reads, e = std::min<int64_t>(n_reads, a + chunk_reads);
        if (offs[e] < offs[a]) return fail(SMEM_E_ARG, "smem_gpu_seed_stream: offsets not ascending");
        max_bases = std::max<uint64_t>(max_bases, offs[e] - offs[a]);
    }
    for (int64_t r = 0; r < n_reads; ++r) {
        if (offs[r + 1] < offs[r]) return fail(SMEM_E_ARG, "smem_gpu_seed_stream: offsets not ascending");
        max_len = std::max<int>(max_len, (int)std::min<uint64_t>(offs[r + 1] - offs[r], 1u << 24));
    }
    if (packed && max_len > SMEM_PINTV_MAX_LEN)
        return fail(SMEM_E_ARG, "smem_gpu_seed_stream: packed entries hold reads up to 8191 bp");
    const int nw = (int)std::max<int64_t>(1, std::min<int64_t>(n_workers, n_chunks));
    const int want_reads = (int)std::min<int64_t>(chunk_reads, std::max<int64_t>(n_reads, 1));
    std::vector<smem_batch_t*> bs(nw, nullptr);
    int rc = SMEM_OK;
    {
        // reuse pooled batches that are large enough (one stream at a time per pool entry)
        std::lock_guard<std::mutex> lk(g->mu);
        for (int w = 0; w < nw; ++w) {
            for (size_t k = 0; k < g->stream_pool.size(); ++k) {
                smem_batch_t* c = g->stream_pool[k];
                if (c->max_reads >= want_reads && c->max_bases >= max_bases && c->max_len >= max_len) {
                    bs[w] = c;
                    g->stream_pool.erase(g->stream_pool.begin() + (long)k);
                    break;
                }
            }
        }
    }
    for (int w = 0; w < nw && rc == SMEM_OK; ++w)
        if (!bs[w]) rc = smem_batch_create(g, want_reads, max_bases, max_len, &bs[w]);
    std::atomic<int64_t> next{0};
    std::atomic<int> err{SMEM_OK};
    std::atomic<uint64_t> n_intv{0}, h2d{0}, d2h{0}, t_stage{0}, t_run{0}, t_fetch{0};
    std::mutex emu;
    std::string emsg;
    // At most `slots` chunks seed at once (SMEM_STREAM_GPU_SLOTS, default 2):
    // two persistent launches overlap each other's tails, as the resident
    // bench's two workers do; a third worker stages / fetches meanwhile
    // instead of queueing a third launch behind them.
    const char* sl_env = getenv("SMEM_STREAM_GPU_SLOTS");
    int slots = sl_env ? std::max(1, atoi(sl_env)) : 2;
    std::mutex slot_mu;
    std::condition_variable slot_cv;
    const auto t0 = std::chrono::steady_clock::now();
    auto worker = [&](int w) {
        smem_batch_t* b = bs[w];
        b->packed = packed;
        for (;;) {
            const int64_t c = next.fetch_add(1);
            if (c >= n_chunks || err.load() != SMEM_OK) break;
            const int64_t a = c * chunk_reads, e = std::min<int64_t>(n_reads, a + chunk_reads);
            const int n = (int)(e - a);
            const auto c0 = std::chrono::steady_clock::now();
            int r = smem_batch_set_reads_packed(b, n, codes, offs + a);
            const auto c1 = std::chrono::steady_clock::now();
            if (!r) {
                {
                    std::unique_lock<std::mutex> lk(slot_mu);
                    slot_cv.wait(lk, [&] { return slots > 0; });
                    --slots;
                }
                r = smem_batch_run(b, opt);
                {
                    std::lock_guard<std::mutex> lk(slot_mu);
                    ++slots;
                }
                slot_cv.notify_one();
            }
            const auto c2 = std::chrono::steady_clock::now();
            if (!r) r = smem_batch_fetch(b);
            const auto c3 = std::chrono::steady_clock::now();
            t_stage += (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(c1 - c0).count();
            t_run += (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(c2 - c1).count();
            t_fetch += (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(c3 - c2).count();
            if (!r) {
                n_intv += b->tot_intv;
                h2d += (offs[e] - offs[a]) + 8ull * (uint64_t)(n + 1);
                d2h += (packed ? 16ull : sizeof(Intv)) * b->tot_intv + 4ull * b->tot_calls + 16ull * (uint64_t)(n + 1);
                if (fn) r = fn(ctx, c, a, n, b);
            }
            if (r) {
                int expect = SMEM_OK;
                if (err.compare_exchange_strong(expect, r)) {
                    std::lock_guard<std::mutex> lk(emu);
                    emsg = g_err;
                }
                break;
            }
        }
    };
    if (rc == SMEM_OK) {
        std::vector<std::thread> th;
        for (int w = 1; w < nw; ++w) th.emplace_back(worker, w);
        worker(0);
        for (auto& t : th) t.join();
        rc = err.load();
    }
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    {
        std::lock_guard<std::mutex> lk(g->mu);
        for (auto* b : bs)
            if (b) {
                b->packed = false;
                // kept for the next call, at most this call's worker count (each
                // pins its staging and result buffers: ~1 GB per 1M-read chunk)
                if (rc == SMEM_OK && !(flags & SMEM_STREAM_RELEASE) && g->stream_pool.size() < (size_t)nw)
                    g->stream_pool.push_back(b);
                else
                    smem_batch_destroy(b);
            }
        // an earlier call's larger pool shrinks to this call's workers
        const size_t keep = (flags & SMEM_STREAM_RELEASE) ? 0 : (size_t)nw;
        while (g->stream_pool.size() > keep) {
            smem_batch_destroy(g->stream_pool.back());
            g->stream_pool.pop_back();
        }
    }
    if (rc != SMEM_OK) {
        if (!emsg.empty()) snprintf(g_err, sizeof(g_err), "smem_gpu_seed_stream: %s", emsg.c_str());
        return rc;
    }
    if (stats) {
        stats->wall_s = secs;
        stats->n_reads = (uint64_t)n_reads;
        stats->n_chunks = (uint64_t)n_chunks;
        stats->n_intv = n_intv.load();
        stats->h2d_bytes = h2d.load();
        stats->d2h_bytes = d2h.load();
        stats->workers = nw;
        stats->stage_s = t_stage.load() * 1e-6;
        stats->run_s = t_run.load() * 1e-6;
        stats->fetch_s = t_fetch.load() * 1e-6;
    }
    return SMEM_OK;
}

// the batch a collect call seeds into: the calling thread's (slot < 0) or the
// worker slot's, (re)created when too small for this batch of reads
static int collect_batch(smem_gpu_t* g, int slot, int n_reads, int max_len, uint64_t bases, smem_batch_t** out) {
    smem_batch_t* b = nullptr;
    std::shared_future<int> res;
    {
        std::lock_guard<std::mutex> lk(g->mu);
        if (slot >= 0 && (size_t)slot < g->reserve.size()) res = g->reserve[(size_t)slot];
    }
    if (res.valid()) res.wait();  // smem_gpu_reserve_slots still sizing this slot
    {
        std::lock_guard<std::mutex> lk(g->mu);
        if (slot >= 0) {
            if ((size_t)slot >= g->slots.size()) g->slots.resize((size_t)slot + 1, nullptr);
            b = g->slots[(size_t)slot];
        } else {
            auto it = g->per_thread.find(std::this_thread::get_id());
            if (it != g->per_thread.end()) b = it->second;
        }
    }
    if (!b || b->max_reads < n_reads || b->max_len < max_len || b->max_bases < bases) {
        const int mr = std::max(n_reads, b ? b->max_reads : 1);
        const int ml = std::max(max_len, b ? b->max_len : 1);
        const uint64_t mb = std::max(bases, b ? b->max_bases : 1);
        smem_batch_t* nb = nullptr;
        int rc = smem_batch_create(g, std::max(mr, 1), std::max<uint64_t>(mb, 1), ml, &nb);
        if (rc) return rc;
        std::lock_guard<std::mutex> lk(g->mu);
        if (b) smem_batch_destroy(b);
        if (slot >= 0) g->slots[(size_t)slot] = nb;
        else g->per_thread[std::this_thread::get_id()] = nb;
        b = nb;
    }
    *out = b;
    return SMEM_OK;
}

// the later stages' scratch of a slot batch, sized before its first use at
// per-read estimates above what 150-250 bp reads need on both bench profiles
// (28-35 intervals, 4.5-10 seed occurrences, ~3 chains and regions per read):
// a worker's first batches then do not reallocate (each reallocation frees,
// and hipFree waits for the whole device).  A batch that needs more grows as
// before.  (Generous estimates cost at shutdown: 16 slots of 62.5k reads at
// 48 / 24 / 8 / 16 per read held 38.6 GB and took 0.43 s to free.)
// (no device work here or in smem_batch_create: smem_gpu_reserve_slots runs
// both once with a measuring Arena, whose buffers are placeholders)
static int batch_prealloc(smem_batch_t* b) {
    const uint64_t R = (uint64_t)b->max_reads;
    const uint64_t ni = R * 40, no = R * 16, nc = R * 6, ns = R * 12;
    HIP_TRY(b->d_flat_intv.ensure(ni));
    HIP_TRY(b->d_flat_calls.ensure(R * 8));
    HIP_TRY(b->d_occ_n.grow(ni));
    HIP_TRY(b->d_occ_off.grow(ni + 1));
    HIP_TRY(b->d_sa_pos.grow(no));
    HIP_TRY(b->d_kstart.grow(no + 2));
    size_t tmp = 0;
    HIP_TRY(smem_launch_offsets(nullptr, nullptr, (int)ni, nullptr, &tmp, nullptr));
    HIP_TRY(b->d_sa_tmp.grow(tmp + 256));
    HIP_TRY(b->d_seed.grow(no));
    HIP_TRY(b->d_next.grow(no));
    HIP_TRY(b->d_chn.grow(no));
    HIP_TRY(b->d_ord.grow(no));
    HIP_TRY(b->d_ord2.grow(no));
    HIP_TRY(b->d_flt.grow(no));
    HIP_TRY(b->d_node.grow(no / 7 + 3 * R + 8));
    HIP_TRY(b->d_n_out.grow(R));
    HIP_TRY(b->d_ns_out.grow(R));
    HIP_TRY(b->d_chain_off.grow(R + 1));
    HIP_TRY(b->d_seed_off.grow(R + 1));
    HIP_TRY(b->d_heavy.grow(2 * R + 4));
    HIP_TRY(b->d_out_chain.grow(nc));
    HIP_TRY(b->d_out_seed.grow(ns));
    HIP_TRY(b->d_aln_srt.grow(ns + 1));
    HIP_TRY(b->d_aln_raw.grow(ns + 1));
    HIP_TRY(b->d_aln_nregs.grow(R));
    HIP_TRY(b->d_aln_regoff.grow(R + 1));
    HIP_TRY(b->d_aln_ctr.grow(smem::ALN_CTRS));
    AlnHeavyBufs& H = b->aln_heavy;
    HIP_TRY(H.pre.grow(ns));
    HIP_TRY(H.pre_ok.grow(ns));
    HIP_TRY(H.span.grow(2 * nc));
    HIP_TRY(H.sdec.grow(nc));
    HIP_TRY(H.tasks.grow(nc));
    HIP_TRY(H.torder.grow(nc));
    HIP_TRY(H.tfail.grow(nc));
    HIP_TRY(H.lq.grow(smem::LQ_WORDS));
    HIP_TRY(H.htasks.grow(ns));
    HIP_TRY(H.htorder.grow(ns));
    HIP_TRY(H.htfail.grow(ns));
    HIP_TRY(H.hlq.grow(smem::LQ_WORDS));
    HIP_TRY(H.chain_read.grow(nc));
    HIP_TRY(H.swlist.grow(nc));
    HIP_TRY(H.short_ok.grow(nc));
    HIP_TRY(H.pre_short.grow(nc));
    HIP_TRY(H.heavy.grow(R));
    HIP_TRY(H.hcnt.grow(R));
    HIP_TRY(H.hscnt.grow(R));
    HIP_TRY(H.hoff.grow(R + 1));
    HIP_TRY(H.rnext.grow(ns));
    {
        // the heavy walk's candidate index (the heavy reads' seeds + chains: ~4 a read
        // human-like, 8 reserved) and the giant split's lists, carved with the rest of the
        // slot: made on a worker's first batch they were ~13 allocations a slot inside
        // mem_process_seqs (and as many hipFree calls at exit)
        const uint64_t mc = R * 8, G = std::min<uint64_t>(R, 2048);
        size_t tb = 0;
        HIP_TRY(smem_launch_offsets(nullptr, nullptr, (int)R, nullptr, &tb, nullptr));
        HIP_TRY(H.tmp.grow(tb + 256));
        HIP_TRY(H.ccnt.grow(R));
        HIP_TRY(H.coff.grow(R + 1));
        HIP_TRY(H.chord.grow(R));
        HIP_TRY(H.ckey.grow(mc));
        HIP_TRY(H.ckey2.grow(mc));
        HIP_TRY(H.cval.grow(mc));
        HIP_TRY(H.cval2.grow(mc));
        HIP_TRY(H.chmax.grow(R));
        HIP_TRY(H.crb.grow(mc));
        HIP_TRY(H.cre.grow(mc));
        HIP_TRY(H.cq.grow(mc));
        HIP_TRY(H.cmade.grow(mc));
        HIP_TRY(H.cpos_s.grow(ns));
        HIP_TRY(H.cpos_c.grow(nc));
        HIP_TRY(H.crng.grow(ns));
        smem::AlnParams P0{};
        smem::CandParams C0{};
        C0.m = mc, C0.n_heavy = (uint32_t)R;
        size_t sb = 0;
        HIP_TRY(smem_launch_aln_cand(&P0, &C0, nullptr, &sb, 1, nullptr));
        HIP_TRY(H.ctmp.grow(sb + 256));
        HIP_TRY(H.heavy2.grow(R));
        HIP_TRY(H.hcnt2.grow(R));
        HIP_TRY(H.hscnt2.grow(R));
        HIP_TRY(H.rgiant.grow(R));
        HIP_TRY(H.gctr.grow(smem::ALN_CTRS));
        HIP_TRY(H.gtasks.grow(ns));
        HIP_TRY(H.gtorder.grow(ns));
        HIP_TRY(H.gtfail.grow(ns));
        HIP_TRY(H.glq.grow(smem::LQ_WORDS));
        HIP_TRY(H.ccnt_g.grow(G));
        HIP_TRY(H.coff_g.grow(G + 1));
        HIP_TRY(H.chord_g.grow(R));
        C0.n_heavy = (uint32_t)G;
        sb = 0;
        HIP_TRY(smem_launch_aln_cand(&P0, &C0, nullptr, &sb, 1, nullptr));
        HIP_TRY(H.ctmp_g.grow(sb + 256));
    }
    // (H.ht, the walk's bin hash, is grown by run_aln only for a walk without the candidate index)
    HIP_TRY(b->d_aln_out.grow(R * 4));
    HIP_TRY(b->h_aln_regoff.grow(R + 1));
    HIP_TRY(b->h_aln_regs.grow(R * 4));  // pinned: the regions fetched (~3 per read)
    if (!b->ev_join) HIP_TRY(hipEventCreateWithFlags(&b->ev_join, hipEventDisableTiming));
    if (!b->ev_fork) HIP_TRY(hipEventCreateWithFlags(&b->ev_fork, hipEventDisableTiming));
    if (!b->ev_giant) HIP_TRY(hipEventCreateWithFlags(&b->ev_giant, hipEventDisableTiming));
    return SMEM_OK;
}

// one pass of every stage over a few reads cut from the resident .pac on a
// slot batch: each kernel's code object is loaded on its first launch, and
// that load should not fall on a worker's first batch
static int batch_warmup(smem_batch_t* b) {
    smem_gpu_t* g = b->g;
    // default: each kernel file's code object loaded by a query, no device
    // work (gpu_open has already done it; a pass of the stages would queue
    // behind the .sa densification) -- SMEM_GPU_WARMUP=full: that pass, over
    // reads cut from the .pac
    const char* wv = getenv("SMEM_GPU_WARMUP");
    if (!(wv && !strcmp(wv, "full"))) {
        HIP_TRY(hipSetDevice(g->device));
        HIP_TRY(smem_preload_seed());
        HIP_TRY(smem_preload_chain());
        HIP_TRY(smem_preload_ksw());
        HIP_TRY(smem_preload_aln());
        return SMEM_OK;
    }
    if (!g->d_pac || g->l_pac < 4096) return SMEM_OK;
    const int nr = std::min(64, b->max_reads), L = std::min(150, b->max_len);
    std::vector<uint8_t> pk((size_t)(L + 8) / 4 + 2), codes((size_t)nr * L);
    std::vector<const uint8_t*> seq((size_t)nr);
    std::vector<int> len((size_t)nr, L);
    for (int r = 0; r < nr; ++r) {
        const uint64_t beg = (uint64_t)(g->l_pac - L - 8) / (uint64_t)nr * (uint64_t)r / 4 * 4;
        HIP_TRY(hipMemcpy(pk.data(), g->d_pac + beg / 4, pk.size(), hipMemcpyDeviceToHost));
        for (int i = 0; i < L; ++i) codes[(size_t)r * L + i] = pk[(size_t)i >> 2] >> ((~i & 3) << 1) & 3;
        seq[(size_t)r] = codes.data() + (size_t)r * L;
    }
    smem_opt_t so;
    smem_chain_opt_t co;
    smem_aln_opt_t ao;
    smem_opt_default(&so);
    smem_chain_opt_default(&co);
    smem_aln_opt_default(&ao);
    int rc = smem_batch_set_reads(b, nr, seq.data(), len.data());
    if (!rc) rc = smem_batch_run(b, &so);
    if (!rc && g->d_sa) rc = smem_batch_sa(b, so.min_seed_len, 10000);
    if (!rc && g->d_sa) rc = smem_batch_chain(b, g->l_pac, &co);
    if (!rc && g->d_sa && b->max_len <= 1024) rc = smem_batch_chain2aln(b, &ao);
    if (!rc && b->aln_ran) rc = smem_batch_fetch_mask(b, SMEM_FETCH_REGS);
    return rc;
}

int smem_batch_memory(const smem_batch_t* b, uint64_t* device_bytes, uint64_t* pinned_bytes) {
    if (!b) return SMEM_E_ARG;
    uint64_t d = 0, h = 0;
    batch_bufs(const_cast<smem_batch_t*>(b), [&](auto& x) { d += x.bytes(); }, [&](auto& x) { h += x.bytes(); });
    if (device_bytes) *device_bytes = d;
    if (pinned_bytes) *pinned_bytes = h;
    return SMEM_OK;
}

int smem_gpu_memory(smem_gpu_t* g, uint64_t* index_bytes, uint64_t* batch_bytes, uint64_t* pinned_bytes, int* n_batches) {
    if (!g) return SMEM_E_ARG;
    gpu_wait(g);
    uint64_t ix = 0, d = 0, h = 0;
    int nb = 0;
    const uint64_t n_ref = (g->bwt_size + 15) / 16;
    ix += (n_ref * 16 + 16) * sizeof(uint32_t);                                   // Occ64
    if (g->d_bwt) ix += (g->bwt_size + 16) * sizeof(uint32_t);                    // reference layout (A/B builds)
    if (g->d_occ192) ix += ((2 * n_ref + 2) / 3 * 16 + 16) * sizeof(uint32_t);
    if (g->d_kt) ix += (((1ull << (2 * (g->kt_k + 1))) - 4) / 3) * 16;
    if (g->d_sa) ix += (g->n_sa + 1) * sizeof(uint64_t);                          // densified SA
    if (g->d_sa_raw) ix += ((g->L2[4] >> 5) + 2) * sizeof(uint64_t);              // the uploaded .sa (sa_intv 32)
    if (g->d_pac) ix += (uint64_t)(g->l_pac + 3) / 4 + 64;
    {
        std::lock_guard<std::mutex> lk(g->mu);
        auto add = [&](const smem_batch_t* b) {
            uint64_t bd = 0, bh = 0;
            if (b && smem_batch_memory(b, &bd, &bh) == SMEM_OK) d += bd, h += bh, ++nb;
        };
        for (auto& kv : g->per_thread) add(kv.second);
        for (auto* b : g->slots) add(b);
        for (auto* b : g->stream_pool) add(b);
        // SMEM_GPU_MEMORY_DETAIL=1: the first slot's device buffers of >= 8 MB, by their place in
        // batch_bufs' visit order (a diagnostic of the per-slot footprint)
        if (getenv("SMEM_GPU_MEMORY_DETAIL") && !g->slots.empty() && g->slots[0]) {
            int k = 0;
            uint64_t mx = 0;
            std::string line;
            batch_bufs(g->slots[0], [&](auto& x) {
                if (x.bytes() >= (8ull << 20)) line += " #" + std::to_string(k) + ":" + std::to_string(x.bytes() >> 20) + "M";
                mx += x.bytes();
                ++k;
            }, [](auto&) {});
            fprintf(stderr, "[M::smem_gpu_memory] device %d slot 0 (max_reads %d): %.3f GB;%s\n", g->device,
                    g->slots[0]->max_reads, mx / 1e9, line.c_str());
        }
    }
    if (index_bytes) *index_bytes = ix;
    if (batch_bytes) *batch_bytes = d;
    if (pinned_bytes) *pinned_bytes = h;
    if (n_batches) *n_batches = nb;
    return SMEM_OK;
}

int smem_gpu_fault(const smem_gpu_t* g, char* msg, int msg_len) {
    if (!g) return SMEM_E_ARG;
    const int f = const_cast<smem_gpu_t*>(g)->faulted.load();
    if (f && msg && msg_len > 0) {
        std::lock_guard<std::mutex> lk(const_cast<smem_gpu_t*>(g)->adm_mu);
        snprintf(msg, (size_t)msg_len, "%s", g->fault_msg);
    }
    return f;
}

int smem_gpu_set_max_active(smem_gpu_t* g, int n) {
    g_err[0] = 0;
    if (!g || n < 0 || n > 256) return fail(SMEM_E_ARG, "smem_gpu_set_max_active: 0..256");
    std::lock_guard<std::mutex> lk(g->adm_mu);
    g->max_active = n > 0 ? n : 8;
    g->adm_cv.notify_all();
    return SMEM_OK;
}

int smem_gpu_get_max_active(const smem_gpu_t* g) {
    if (!g) return SMEM_E_ARG;
    std::lock_guard<std::mutex> lk(const_cast<smem_gpu_t*>(g)->adm_mu);
    return g->max_active;
}

int smem_gpu_reserve_slots(smem_gpu_t* g, int n_slots, int reads_per_slot, int max_len) {
    g_err[0] = 0;
    if (!g || n_slots <= 0 || n_slots > 4096 || reads_per_slot <= 0 || max_len <= 0 || max_len > (1 << 24) ||
        (uint64_t)reads_per_slot * (uint64_t)max_len >= (1ull << 32) - 64)
        return fail(SMEM_E_ARG, "smem_gpu_reserve_slots");
    if (int r = gpu_check(g)) return r;
    std::lock_guard<std::mutex> lk(g->mu);
    for (auto& f : g->reserve)
        if (f.valid() && f.wait_for(std::chrono::seconds(0)) != std::future_status::ready)
            return fail(SMEM_E_ARG, "smem_gpu_reserve_slots: a reservation is still running");
    // one host thread per slot (as the workers would each create their own on
    // first use), slot 0's also runs the warm-up; a worker waits for its own
    // slot only
    g->reserve.assign((size_t)n_slots, std::shared_future<int>());
    for (int k = 0; k < n_slots; ++k)
        g->reserve[(size_t)k] = std::async(std::launch::async, [g, k, reads_per_slot, max_len]() -> int {
            g_no_inject = 1;
            if (hipSetDevice(g->device) != hipSuccess) return SMEM_E_DEVICE;
            const auto t0 = std::chrono::steady_clock::now();
            const uint64_t bases = (uint64_t)reads_per_slot * (uint64_t)max_len;
            // the slot's buffers from two blocks (Arena): the same calls once
            // to measure, then to carve (SMEM_GPU_ARENA=0: one allocation each)
            Arena ad, ah;
            const char* av = getenv("SMEM_GPU_ARENA");
            if (!(av && atoi(av) == 0)) {
                Arena md, mh;
                md.measure = mh.measure = true;
                t_dev_arena = &md, t_host_arena = &mh;
                smem_batch_t* m = nullptr;
                int r = smem_batch_create(g, reads_per_slot, bases, max_len, &m);
                if (r == SMEM_OK) r = batch_prealloc(m);
                t_dev_arena = t_host_arena = nullptr;
                if (m) smem_batch_destroy(m);
                if (r == SMEM_OK && hipMalloc(&ad.base, md.used) == hipSuccess) ad.cap = md.used;
                if (r == SMEM_OK && hipHostMalloc(reinterpret_cast<void**>(&ah.base), mh.used, hipHostMallocDefault) ==
                                        hipSuccess)
                    ah.cap = mh.used;
                t_dev_arena = ad.base ? &ad : nullptr, t_host_arena = ah.base ? &ah : nullptr;
            }
            smem_batch_t* b = nullptr;
            int rc = smem_batch_create(g, reads_per_slot, bases, max_len, &b);
            const auto t1 = std::chrono::steady_clock::now();
            if (rc == SMEM_OK) rc = batch_prealloc(b);
            t_dev_arena = t_host_arena = nullptr;
            if (b) {
                b->arena_dev = ad.base, b->arena_host = ah.base;
            } else {  // smem_batch_create failed and released what it carved
                if (ad.base) (void)hipFree(ad.base);
                if (ah.base) (void)hipHostFree(ah.base);
            }
            const auto t2 = std::chrono::steady_clock::now();
            if (rc == SMEM_OK && k == 0) rc = batch_warmup(b);
            if (getenv("SMEM_GPU_TIMES")) {  // diagnostics, as the binding's per-batch times
                const auto t3 = std::chrono::steady_clock::now();
                auto sec = [](std::chrono::steady_clock::duration d) { return std::chrono::duration<double>(d).count(); };
                fprintf(stderr, "[M::smem_gpu_reserve_slots] device %d slot %d at %.3f s: create %.4f s, stage scratch "
                        "%.4f s, warm-up %.4f s (rc %d)\n", g->device, k,
                        std::chrono::duration<double>(t0.time_since_epoch()).count() - g_t_lib, sec(t1 - t0),
                        sec(t2 - t1), sec(t3 - t2), rc);
            }
            if (rc != SMEM_OK) {  // the slot is created on its first use, as without the reservation
                smem_batch_destroy(b);
                return rc;
            }
            std::lock_guard<std::mutex> lk2(g->mu);
            if (g->slots.size() <= (size_t)k) g->slots.resize((size_t)k + 1, nullptr);
            if (g->slots[(size_t)k]) smem_batch_destroy(g->slots[(size_t)k]);
            g->slots[(size_t)k] = b;
            return SMEM_OK;
        }).share();
    return SMEM_OK;
}

int smem_gpu_collect_ex(smem_gpu_t* g, int slot, int n_reads, const uint8_t* const* seq, const int* len,
                        const smem_opt_t* opt, int flags, smem_batch_t** batch_out) {
    g_err[0] = 0;
    if (!g || !opt || !batch_out || n_reads < 0 || (n_reads > 0 && (!seq || !len)) || slot > 4096 ||
        (flags & ~SMEM_COLLECT_NO_FETCH))
        return fail(SMEM_E_ARG, "smem_gpu_collect");
    *batch_out = nullptr;
    int max_len = 1;
    uint64_t bases = 0;
    for (int i = 0; i < n_reads; ++i) {
        if (len[i] < 0) return fail(SMEM_E_ARG, "smem_gpu_collect: negative length");
        max_len = std::max(max_len, len[i]);
        bases += (uint64_t)len[i];
    }
    smem_batch_t* b = nullptr;
    static const bool times = getenv("SMEM_GPU_TIMES") != nullptr;
    const double t0 = times ? now_s() : 0;
    g_t_ready = g_t_admit = 0;
    int rc = collect_batch(g, slot, n_reads, max_len, bases, &b);
    const double t1 = times ? now_s() : 0;
    if (!rc) rc = smem_batch_set_reads(b, n_reads, seq, len);
    const double t2 = times ? now_s() : 0;
    if (!rc) rc = smem_batch_run(b, opt);
    if (!rc && !(flags & SMEM_COLLECT_NO_FETCH)) rc = smem_batch_fetch(b);
    if (times)  // diagnostics: where a worker's seeding call spent its time
        fprintf(stderr, "[M::smem_gpu_collect] slot %d at %.3f s: batch %.4f s, reads in %.4f s, seeding %.4f s "
                "(device-ready waits %.4f s, admission waits %.4f s)\n", slot, t0 - g_t_lib, t1 - t0, t2 - t1,
                now_s() - t2, g_t_ready, g_t_admit);
    if (!rc) *batch_out = b;
    return rc;
}

int smem_gpu_collect(smem_gpu_t* g, int n_reads, const uint8_t* const* seq, const int* len, const smem_opt_t* opt,
                     smem_batch_t** batch_out) {
    return smem_gpu_collect_ex(g, -1, n_reads, seq, len, opt, 0, batch_out);
}

int smem_gpu_parse_devices(const char* spec, int* devices, int max_devices) {
    g_err[0] = 0;
    if (!devices || max_devices <= 0) return fail(SMEM_E_ARG, "smem_gpu_parse_devices");
    const int n_vis = smem_gpu_device_count();
    if (!spec || !*spec) {  // every visible device
        if (n_vis <= 0) return fail(SMEM_E_DEVICE, "smem_gpu_parse_devices: no HIP device");
        const int n = std::min(n_vis, max_devices);
        for (int i = 0; i < n; ++i) devices[i] = i;
        return n;
    }
    int n = 0;
    const char* p = spec;
    while (*p) {
        char* e = nullptr;
        const long v = strtol(p, &e, 10);
        if (e == p || v < 0 || v > 1 << 20) return fail(SMEM_E_ARG, "smem_gpu_parse_devices: bad device list");
        if (n == max_devices) return fail(SMEM_E_ARG, "smem_gpu_parse_devices: too many devices");
        devices[n++] = (int)v;
        p = e;
        if (*p == ',' && p[1]) ++p;
        else if (*p) return fail(SMEM_E_ARG, "smem_gpu_parse_devices: bad device list");
    }
    if (n == 0) return fail(SMEM_E_ARG, "smem_gpu_parse_devices: empty device list");
    return n;
}

int smem_gpu_init_devices(smem_gpu_t** gpus, int n, const int* devices, const uint32_t* bwt, uint64_t bwt_size,
                          uint64_t primary, const uint64_t L2[5], const smem_sa_t* sa, const uint8_t* pac,
                          int64_t l_pac) {
    g_err[0] = 0;
    if (!gpus || n <= 0 || n > 1024) return fail(SMEM_E_ARG, "smem_gpu_init_devices");
    for (int i = 0; i < n; ++i) gpus[i] = nullptr;
    std::vector<int> rc(n, SMEM_OK);
    std::vector<std::string> msg(n);
    // one host thread per device: the uploads (and each device's Occ64 /
    // .sa densification kernels) run side by side
    auto open1 = [&](int i) {
        smem_gpu_t* g = nullptr;
        const auto t0 = std::chrono::steady_clock::now();
        int r = smem_gpu_init(&g, devices ? devices[i] : i, bwt, bwt_size, primary, L2);
        const auto t1 = std::chrono::steady_clock::now();
        if (!r && sa) r = smem_gpu_load_sa(g, sa);
        const auto t2 = std::chrono::steady_clock::now();
        if (!r && pac) r = smem_gpu_load_pac(g, pac, l_pac);
        if (getenv("SMEM_GPU_TIMES")) {
            auto sec = [](std::chrono::steady_clock::duration d) { return std::chrono::duration<double>(d).count(); };
            fprintf(stderr, "[M::smem_gpu_init_devices] device %d: index upload + Occ64 %.4f s, .sa upload %.4f s, "
                    ".pac upload %.4f s (rc %d)\n", devices ? devices[i] : i, sec(t1 - t0), sec(t2 - t1),
                    sec(std::chrono::steady_clock::now() - t2), r);
        }
        if (r) {
            msg[i] = g_err;
            smem_gpu_shutdown(g);
            g = nullptr;
        }
        rc[i] = r;
        gpus[i] = g;
    };
    std::vector<std::thread> th;
    for (int i = 1; i < n; ++i) th.emplace_back(open1, i);
    open1(0);
    for (auto& t : th) t.join();
    for (int i = 0; i < n; ++i) {
        if (rc[i] == SMEM_OK) continue;
        for (int k = 0; k < n; ++k) {
            smem_gpu_shutdown(gpus[k]);
            gpus[k] = nullptr;
        }
        snprintf(g_err, sizeof(g_err), "smem_gpu_init_devices: device %d: %s", devices ? devices[i] : i, msg[i].c_str());
        return rc[i];
    }
    return SMEM_OK;
}

// the device work of a handle as a chain of background steps: each waits for
// the one before; a failure faults the handle (3), later steps do nothing
static void gpu_chain(smem_gpu_t* g, const char* what, std::function<int()> step) {
    std::lock_guard<std::mutex> lk(g->ready_mu);
    std::shared_future<int> prev = g->ready;
    g->ready = std::async(std::launch::async, [g, what, prev, step]() -> int {
        if (prev.valid() && prev.get() != SMEM_OK) return SMEM_E_DEVICE;
        const auto t0 = std::chrono::steady_clock::now();
        g_hip_fault = 0;  // this thread's: set by fail() on a runtime error that breaks the device
        const int r = step();
        if (getenv("SMEM_GPU_TIMES"))
            fprintf(stderr, "[M::smem_gpu_async] device %d: %s %.4f s, done at %.3f s (rc %d)\n", g->device, what,
                    std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(), now_s() - g_t_lib, r);
        if (r) {  // every call on the handle is refused from now on (SMEM_E_DEVICE): the caller's CPU path
            std::lock_guard<std::mutex> lk(g->adm_mu);
            snprintf(g->fault_msg, sizeof(g->fault_msg), "initialisation failed: %s", g_err);
            // a HIP runtime failure (1, as during a run: its diagnostics may have reached stdout)
            // or a refusal such as an allocation that does not fit (3)
            g->faulted.store(g_hip_fault == 1 ? 1 : 3);
        }
        return r;
    }).share();
}

// SMEM_GPU_CRASH_TRACE=1 (diagnostics): a host SIGSEGV / SIGBUS / SIGFPE / SIGABRT prints the
// faulting thread's backtrace (module + offset, resolved offline with addr2line) and the
// executable mappings of the program and this library to stderr, then takes the default action
static char g_crash_maps[1 << 20];
static void crash_trace(int sig, siginfo_t* si, void*) {
    char buf[160];
    int n = snprintf(buf, sizeof buf, "[smem crash] signal %d at %p, thread %ld\n", sig, si ? si->si_addr : nullptr,
                     (long)syscall(SYS_gettid));
    if (write(2, buf, (size_t)n) < 0) {}
    void* fr[64];
    backtrace_symbols_fd(fr, backtrace(fr, 64), 2);
    const int fd = open("/proc/self/maps", O_RDONLY);
    if (fd >= 0) {
        size_t m = 0;
        ssize_t r;
        while (m < sizeof g_crash_maps - 1 && (r = read(fd, g_crash_maps + m, sizeof g_crash_maps - 1 - m)) > 0)
            m += (size_t)r;
        close(fd);
        g_crash_maps[m] = 0;
        for (char* l = g_crash_maps; *l;) {
            char* e = strchr(l, '\n');
            const size_t len = e ? (size_t)(e - l + 1) : strlen(l);
            const char save = l[len];
            l[len] = 0;
            if (strstr(l, "r-xp") && (strstr(l, "bwa") || strstr(l, "smemgpu")))
                if (write(2, l, len) < 0) {}
            l[len] = save;
            l += len;
        }
    }
    signal(sig, SIG_DFL);
    raise(sig);
}

static void crash_trace_install() {
    static std::once_flag once;
    std::call_once(once, [] {
        const char* e = getenv("SMEM_GPU_CRASH_TRACE");
        if (!e || !atoi(e)) return;
        void* fr[4];
        (void)backtrace(fr, 4);  // libgcc loaded now, not inside the handler
        struct sigaction sa;
        memset(&sa, 0, sizeof sa);
        sa.sa_sigaction = crash_trace;
        sa.sa_flags = SA_SIGINFO | SA_RESETHAND;
        for (int sg : {SIGSEGV, SIGBUS, SIGFPE, SIGABRT}) sigaction(sg, &sa, nullptr);
    });
}

int smem_gpu_open_async(smem_gpu_t** out, int device, const uint32_t* bwt, uint64_t bwt_size, uint64_t primary,
                        const uint64_t L2[5]) {
    crash_trace_install();
    g_err[0] = 0;
    if (!out || !bwt || bwt_size < 16 || !L2) return fail(SMEM_E_ARG, "smem_gpu_open_async: bad index");
    *out = nullptr;
    if (L2[4] >= (1ull << 34) - 2) return fail(SMEM_E_ARG, "smem_gpu_open_async: seq_len >= 2^34 not supported");
    if ((bwt_size + 16) * sizeof(uint32_t) > (1ull << 32))
        return fail(SMEM_E_ARG, "smem_gpu_open_async: index larger than 4 GiB not supported");
    int nv = 0;  // the device exists (reported here, before anything runs)
    if (hipGetDeviceCount(&nv) != hipSuccess || nv <= 0) return fail(SMEM_E_DEVICE, "smem_gpu_open_async: no HIP device");
    if (device < 0 || device >= nv) return fail(SMEM_E_ARG, "smem_gpu_open_async: device out of range");
    smem_gpu_t* g = gpu_handle(device, bwt_size, primary, L2);
    if (!g) return fail(SMEM_E_NOMEM, "smem_gpu_open_async");
    gpu_chain(g, "index upload + Occ64", [g, bwt]() { return gpu_open(g, bwt); });
    *out = g;
    return SMEM_OK;
}

int smem_gpu_load_sa_async(smem_gpu_t* g, const smem_sa_t* sa) {
    g_err[0] = 0;
    if (!g || !sa || !sa->sa || sa->n_sa == 0 || sa->sa_intv == 0 || (sa->sa_intv & (sa->sa_intv - 1)) ||
        sa->seq_len != g->L2[4] || sa->n_sa != (sa->seq_len + sa->sa_intv) / sa->sa_intv || sa->primary != g->primary)
        return fail(SMEM_E_ARG, "smem_gpu_load_sa_async: SA does not belong to this index");
    const smem_sa_t copy = *sa;  // the caller's struct may go out of scope; its array may not
    gpu_chain(g, ".sa upload (+ densify launched)", [g, copy]() { return load_sa_impl(g, &copy); });
    return SMEM_OK;
}

int smem_gpu_load_pac_async(smem_gpu_t* g, const uint8_t* pac, int64_t l_pac) {
    g_err[0] = 0;
    if (!g || !pac || l_pac <= 0 || 2 * (uint64_t)l_pac != g->L2[4])
        return fail(SMEM_E_ARG, "smem_gpu_load_pac_async: pac does not belong to this index");
    gpu_chain(g, ".pac upload", [g, pac, l_pac]() { return load_pac_impl(g, pac, l_pac); });
    return SMEM_OK;
}

int smem_gpu_init_devices_async(smem_gpu_t** gpus, int n, const int* devices, const uint32_t* bwt, uint64_t bwt_size,
                                uint64_t primary, const uint64_t L2[5], const smem_sa_t* sa, const uint8_t* pac,
                                int64_t l_pac) {
    g_err[0] = 0;
    if (!gpus || n <= 0 || n > 1024) return fail(SMEM_E_ARG, "smem_gpu_init_devices_async");
    for (int i = 0; i < n; ++i) gpus[i] = nullptr;
    int rc = SMEM_OK;
    for (int i = 0; i < n && rc == SMEM_OK; ++i) {
        rc = smem_gpu_open_async(&gpus[i], devices ? devices[i] : i, bwt, bwt_size, primary, L2);
        if (rc == SMEM_OK && sa) rc = smem_gpu_load_sa_async(gpus[i], sa);
        if (rc == SMEM_OK && pac) rc = smem_gpu_load_pac_async(gpus[i], pac, l_pac);
    }
    if (rc != SMEM_OK) {
        std::string msg = g_err;
        for (int k = 0; k < n; ++k) {
            smem_gpu_shutdown(gpus[k]);
            gpus[k] = nullptr;
        }
        snprintf(g_err, sizeof(g_err), "smem_gpu_init_devices_async: %s", msg.c_str());
    }
    return rc;
}

int smem_gpu_wait_ready(smem_gpu_t* g) {
    g_err[0] = 0;
    if (!g) return fail(SMEM_E_ARG, "smem_gpu_wait_ready");
    gpu_wait(g);  // the upload chain
    std::vector<std::shared_future<int>> res;
    {
        std::lock_guard<std::mutex> lk(g->mu);
        res = g->reserve;
    }
    for (auto& f : res)  // the worker slots being sized (smem_gpu_reserve_slots)
        if (f.valid()) f.wait();
    if (int r = gpu_check(g)) return r;
    if (g->sa_ready) {  // the .sa densification on the init stream (batches do not
        HIP_TRY(hipSetDevice(g->device));  // need it: their lookups use the uploaded
        HIP_TRY(hipEventSynchronize(g->sa_ready));  // samples until it is done)
        HIP_TRY(release_link(g, true));
        HIP_TRY(trim_default_pool(g));
        sa_check(g);
    }
    return SMEM_OK;
}

}  // extern "C"
