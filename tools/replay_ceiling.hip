// replay_ceiling.hip -- the request ceiling of the seeding kernel's OWN
// access stream: every Occ64 bucket load the kernel makes for a sample of the
// bench's reads (oracle/smem_oracle.c orc_seed_trace, in extend order per
// read), replayed with nothing else in the way.
//
// tools/gather_ceiling.hip measures uniformly random 32-B buckets at 12 waves
// per CU; the kernel runs 15 waves per CU (960 lanes) and its stream is not
// uniform: short strings hit a few hot buckets (L2 / MALL hits), so against
// that ceiling the uniform profile came out above 1.  Here a
// persistent grid of W waves per CU replays the recorded stream: each lane
// takes one read's extends in order (claimed from a counter, one atomic per
// wave), issues each extend's one or two 32-B buckets (2 x 16-B loads each, as
// the kernel does) and waits for them (vmcnt(0)) before its next extend -- 64
// independent dependency chains per wave, the wp kernel's shape (every lane an
// extend per iteration).  The trace words themselves stream through a 2-window
// prefetch (4 words per 16-B load, one window ahead).  Reads are replayed
// `reps` times (replica k of read r claimed ~k x n_reads later: far beyond any
// cache's reuse distance).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/replay_ceiling tools/replay_ceiling.hip
//   tools/replay_ceiling <trace.bin> <table_buckets> <waves_per_cu> [reps=4] [uniform=0]
//
// trace.bin: u64 n_reads, u64 n_loads, u64 read_off[n_reads + 1], u32 loads[n_loads]
// (bit 31 of a load: the second bucket of the same extend).  uniform=1 replaces
// every bucket index by a hash of it (the same count, structure and chains, but
// uniformly spread: the random-gather ceiling at the same occupancy).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

__device__ __forceinline__ uint32_t word(const uint4& w, uint32_t k) {
    return k == 0 ? w.x : k == 1 ? w.y : k == 2 ? w.z : w.w;
}

// loads: padded with 8 zero words past n_loads (the window prefetch reads ahead)
__global__ __launch_bounds__(256) void replay(const uint4* __restrict__ tab, uint64_t n_buckets,
                                              const uint32_t* __restrict__ loads, const uint64_t* __restrict__ roff,
                                              uint64_t n_reads, uint64_t n_items, uint32_t* __restrict__ head,
                                              uint32_t* __restrict__ sink, int uniform,
                                              unsigned long long* __restrict__ n_done) {
    const int lane = threadIdx.x & 63;
    uint64_t cur = 0, end = 0, wbase = 0;
    uint4 win = {0, 0, 0, 0}, nwin = {0, 0, 0, 0};
    bool done = false;
    uint32_t acc = 0;
    unsigned long long cnt = 0;
    for (;;) {
        // lanes whose read ended claim the next (one atomic per wave)
        const bool want = !done && cur >= end;
        const uint64_t m = __ballot(want);
        if (m) {
            const int lead = __builtin_ffsll((long long)m) - 1;
            uint32_t base = 0;
            if (lane == lead) base = atomicAdd(head, (uint32_t)__popcll(m));
            base = (uint32_t)__shfl((int)base, lead);
            if (want) {
                const uint64_t it = base + (uint64_t)__popcll(m & ((1ull << lane) - 1));
                if (it >= n_items) {
                    done = true;
                } else {
                    const uint64_t r = it % n_reads;
                    cur = roff[r], end = roff[r + 1];
                    wbase = cur & ~3ull;
                    win = *reinterpret_cast<const uint4*>(loads + wbase);
                    nwin = *reinterpret_cast<const uint4*>(loads + wbase + 4);
                }
            }
        }
        if (__ballot(!done) == 0) break;
        const bool act = !done && cur < end;
        uint32_t b0 = 0, b1 = 0;
        bool two = false;
        if (act) {
            if (cur >= wbase + 4) {  // the window moves on; its successor was loaded an iteration ago
                win = nwin;
                wbase += 4;
                nwin = *reinterpret_cast<const uint4*>(loads + wbase + 4);
            }
            const uint32_t k = (uint32_t)(cur - wbase);
            b0 = word(win, k);
            const uint32_t v1 = k < 3 ? word(win, k + 1) : nwin.x;
            two = cur + 1 < end && (v1 >> 31);
            b1 = v1 & 0x7fffffffu;
            b0 &= 0x7fffffffu;
            if (uniform) b0 = mix(b0 * 2654435761u + 17u), b1 = mix(b1 * 2654435761u + 29u);
            b0 = (uint32_t)(b0 % n_buckets);
            b1 = (uint32_t)(b1 % n_buckets);
        }
        uint4 a0 = {0, 0, 0, 0}, a1 = {0, 0, 0, 0}, c0 = {0, 0, 0, 0}, c1 = {0, 0, 0, 0};
        if (act) {
            a0 = tab[(uint64_t)b0 * 2];
            a1 = tab[(uint64_t)b0 * 2 + 1];
            if (two) {
                c0 = tab[(uint64_t)b1 * 2];
                c1 = tab[(uint64_t)b1 * 2 + 1];
            }
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the extend's buckets (and the window) landed
        acc ^= a0.x ^ a1.w ^ c0.y ^ c1.z;
        if (act) {
            cnt += two ? 2 : 1;
            cur += two ? 2 : 1;
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
    // loads per wave, summed
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor((long long)cnt, o);
    if (lane == 0) atomicAdd(n_done, cnt);
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s trace.bin table_buckets waves_per_cu [reps] [uniform]\n", argv[0]);
        return 2;
    }
    FILE* fp = fopen(argv[1], "rb");
    if (!fp) return 2;
    uint64_t hdr[2];
    if (fread(hdr, 8, 2, fp) != 2) return 2;
    const uint64_t n_reads = hdr[0], n_loads = hdr[1];
    std::vector<uint64_t> roff(n_reads + 1);
    std::vector<uint32_t> loads(n_loads + 8, 0u);
    if (fread(roff.data(), 8, n_reads + 1, fp) != n_reads + 1) return 2;
    if (fread(loads.data(), 4, n_loads, fp) != n_loads) return 2;
    fclose(fp);
    const uint64_t n_buckets = strtoull(argv[2], nullptr, 10);
    const int wpc = atoi(argv[3]);
    const int reps = argc > 4 ? atoi(argv[4]) : 4;
    const int uniform = argc > 5 ? atoi(argv[5]) : 0;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    uint4* tab;
    uint32_t *dl, *head, *sink;
    uint64_t* droff;
    unsigned long long* n_done;
    CHECK(hipMalloc(&tab, n_buckets * 32 + 64));
    CHECK(hipMemset(tab, 1, n_buckets * 32 + 64));
    CHECK(hipMalloc(&dl, loads.size() * 4));
    CHECK(hipMemcpy(dl, loads.data(), loads.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMalloc(&droff, roff.size() * 8));
    CHECK(hipMemcpy(droff, roff.data(), roff.size() * 8, hipMemcpyHostToDevice));
    CHECK(hipMalloc(&head, 4));
    CHECK(hipMalloc(&sink, 4));
    CHECK(hipMalloc(&n_done, 8));
    const int grid = prop.multiProcessorCount * wpc / 4;
    const uint64_t n_items = n_reads * (uint64_t)reps;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int rep = 0; rep < 3; ++rep) {
        CHECK(hipMemset(head, 0, 4));
        CHECK(hipMemset(n_done, 0, 8));
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(replay, dim3(grid), dim3(256), 0, 0, tab, n_buckets, dl, droff, n_reads, n_items, head, sink,
                           uniform, n_done);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        unsigned long long nd = 0;
        CHECK(hipMemcpy(&nd, n_done, 8, hipMemcpyDeviceToHost));
        printf("{\"waves_per_cu\": %d, \"uniform\": %d, \"reads\": %llu, \"bucket_loads\": %llu, \"ms\": %.3f, "
               "\"Gbuckets_per_s\": %.2f, \"loads_per_read\": %.1f, \"n_buckets\": %llu}\n",
               wpc, uniform, (unsigned long long)n_items, nd, ms, nd / ms * 1e-6, (double)nd / (double)n_items,
               (unsigned long long)n_buckets);
        fflush(stdout);
    }
    return 0;
}
