// qe_runtime.hip -- libqe context, caching HBM allocator, lookback state, profiling, the
// relation loader (reference src/utilities.c:105-162) and the on-device splitmix64 generator.
#include <algorithm>
#include <chrono>
#include <cstring>
#include <thread>
#include <vector>

#include "qe_device.h"
#include "qe_internal.h"

namespace qe {

// ---------------------------------------------------------------------------------------------
// allocator: exact size classes (rounded), blocks reused in stream order on the ctx's single
// stream, so no hipMalloc/hipFree inside a steady-state query (cdna_hip_programming.md G9)
// ---------------------------------------------------------------------------------------------
static size_t round_size(size_t b) {
    if (b < 256) return 256;
    if (b <= (64u << 20)) {
        size_t p = 256;
        while (p < b) p <<= 1;
        // quarter steps between powers of two keep waste under 25 %
        size_t q = p >> 2;
        size_t r = ((b + q - 1) / q) * q;
        return r;
    }
    const size_t g = 32u << 20;
    return ((b + g - 1) / g) * g;
}

// placement knobs for A/Bs: QE_ALLOC_PAD=B offsets every new block of >= 16 MiB
// by B bytes inside a larger hipMalloc (the base kept for hipFree); QE_ALLOC_LOG=1 prints each new
// large block's address
static size_t alloc_pad() {
    static const size_t v = [] {
        const char* e = getenv("QE_ALLOC_PAD");
        return e ? (size_t)strtoull(e, nullptr, 0) : (size_t)0;
    }();
    return v;
}
bool alloc_log_on() {
    static const bool v = [] {
        const char* e = getenv("QE_ALLOC_LOG");
        return e && *e == '1';
    }();
    return v;
}
static hipError_t hmalloc(qe_ctx* c, void** p, size_t sz) {
    const size_t pad = sz >= (16u << 20) ? alloc_pad() : 0;
    void* b = nullptr;
    hipError_t e = hipMalloc(&b, sz + pad + DALLOC_SLACK);
    if (e != hipSuccess) return e;
    *p = (char*)b + pad;
    if (pad) c->pad_base[*p] = b;
    if (alloc_log_on() && sz >= (16u << 20))
        fprintf(stderr, "[qe alloc] %zu MiB at %p (base %p)\n", sz >> 20, *p, b);
    return e;
}
static void hfree(qe_ctx* c, void* p) {
    auto it = c->pad_base.find(p);
    if (it != c->pad_base.end()) {
        p = it->second;
        c->pad_base.erase(it);
    }
    (void)hipFree(p);
}

void* dalloc(qe_ctx* c, size_t bytes) {
    size_t sz = round_size(bytes);
    auto it = c->free_blocks.lower_bound(sz);
    if (it != c->free_blocks.end() && it->first <= sz + sz / 8) {
        void* p = it->second;
        size_t got = it->first;
        c->free_blocks.erase(it);
        c->cached -= got;
        c->live[p] = got;
        c->in_use += got;
        return p;
    }
    void* p = nullptr;
    hipError_t e = hmalloc(c, &p, sz);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        // release the cache and retry once
        QE_HIP(hipStreamSynchronize(c->stream));
        for (auto& kv : c->free_blocks) hfree(c, kv.second);
        c->free_blocks.clear();
        c->cached = 0;
        e = hmalloc(c, &p, sz);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            throw Error(QE_ENOMEM, "hipMalloc(" + std::to_string(sz) + ") failed");
        }
    }
    c->live[p] = sz;
    c->in_use += sz;
    return p;
}

void dfree(qe_ctx* c, void* p) {
    if (!p) return;
    // a shared sort's buffer (pinned while this lane reads it) is never recycled: the violation is
    // recorded -- dfree runs inside destructors and qe_pairs_free, where a throw would terminate --
    // and qe_sort_cache(ctx, 0) fails the batch with it
    if (!c->pinned.empty() && c->pinned.count(p)) {
        if (c->late_err.empty()) c->late_err = "internal: dfree of a shared sort's buffer";
        return;
    }
    if (c->hold_frees) {   // two streams in flight: recycled once they have met (SideFork::join)
        c->held.push_back(p);
        return;
    }
    auto it = c->live.find(p);
    if (it == c->live.end()) return;   // not ours (e.g. a relation column)
    size_t sz = it->second;
    c->live.erase(it);
    c->in_use -= sz;
    c->free_blocks.emplace(sz, p);
    c->cached += sz;
}

void drop_partitions(qe_ctx* c) {
    if (c->bparts.empty()) return;
    QE_HIP(hipStreamSynchronize(c->stream));
    for (auto& kv : c->bparts) {
        dfree(c, kv.second.key);
        dfree(c, kv.second.val);
    }
    c->bparts.clear();
    c->bparts_n = c->bparts_p = 0;
}

// ---- the side stream (SideFork): one join side's sort queued beside the other's -------------------
static void swap_state(qe_ctx* c) {
    StreamState& s = c->side;
    std::swap(c->stream, s.stream);
    std::swap(c->lb_status, s.lb_status);
    std::swap(c->lb_status_words, s.lb_status_words);
    std::swap(c->lb_tickets, s.lb_tickets);
    std::swap(c->lb_epoch, s.lb_epoch);
    std::swap(c->d_scratch, s.d_scratch);
    std::swap(c->d_zhist, s.d_zhist);
    std::swap(c->zhist_dirty, s.zhist_dirty);
    std::swap(c->h_scratch, s.h_scratch);
    std::swap(c->wait_ev, s.wait_ev);
    std::swap(c->h_ret, s.h_ret);
    std::swap(c->d_ret, s.d_ret);
    std::swap(c->ret_seq, s.ret_seq);
    c->side_in = !c->side_in;
}

bool side_stream_on() {
    // QE_SIDE_STREAM=1: on.  Off by default: C3 6.30 -> 6.15 / 6.29 -> 5.93 ms per query on two
    // boxes (-2.4 / -5.8 %, profiles/r06d_c3_bench.log, r06e_c3_bench.log; bench.py reports it as
    // `two_stream_sorts`), but the two sides' kernels then share the GPU, so a launch's
    // duration no longer measures that kernel alone -- the line's per-launch roofline would not mean
    // what it says (sort_pass_carry 3.05 -> 4.22 ms of overlapped launch time per query)
    const char* s = getenv("QE_SIDE_STREAM");   // (read per join: tests switch it)
    return s && s[0] == '1';
}

SideFork::SideFork(qe_ctx* cc, bool want) : c(cc) {
    if (!want || !side_stream_on() || c->side_in || c->hold_frees) return;   // (no nesting)
    StreamState& s = c->side;
    if (!s.stream) {   // made once per ctx, on first use
        QE_HIP(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
        QE_HIP(hipMalloc(&s.lb_tickets, LB_MAX_COUNTERS * sizeof(uint32_t)));
        QE_HIP(hipMemsetAsync(s.lb_tickets, 0, LB_MAX_COUNTERS * sizeof(uint32_t), s.stream));
        QE_HIP(hipMalloc(&s.d_scratch, 64 * sizeof(uint64_t)));
        QE_HIP(hipHostMalloc((void**)&s.h_scratch, 64 * sizeof(uint64_t), hipHostMallocDefault));
        for (auto& e : c->fork_ev) QE_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    // the side stream starts after everything queued on the ctx stream so far (its inputs)
    QE_HIP(hipEventRecord(c->fork_ev[0], c->stream));
    QE_HIP(hipStreamWaitEvent(s.stream, c->fork_ev[0], 0));
    c->hold_frees++;
    on = true;
}

void SideFork::enter() {
    if (on && !c->side_in) swap_state(c);
}

void SideFork::leave() {
    if (on && c->side_in) swap_state(c);
}

void SideFork::join() {
    if (!on) return;
    leave();
    on = false;
    // the ctx stream goes on after the side stream's work; then both streams' frees are safe
    QE_HIP(hipEventRecord(c->fork_ev[1], c->side.stream));
    QE_HIP(hipStreamWaitEvent(c->stream, c->fork_ev[1], 0));
    if (--c->hold_frees == 0) {
        std::vector<void*> h;
        h.swap(c->held);
        for (void* p : h) dfree(c, p);
    }
}

SideFork::~SideFork() {
    if (!on) return;
    try {
        join();
    } catch (...) {   // (a failed event call: wait for both streams instead)
        if (c->side_in) swap_state(c);
        (void)hipStreamSynchronize(c->side.stream);
        (void)hipStreamSynchronize(c->stream);
        if (--c->hold_frees == 0) {
            std::vector<void*> h;
            h.swap(c->held);
            for (void* p : h) dfree(c, p);
        }
    }
}

LBSlot lb_acquire(qe_ctx* c, size_t words) {
    if (words > c->lb_status_words) {
        if (c->lb_status) {
            QE_HIP(hipStreamSynchronize(c->stream));
            QE_HIP(hipFree(c->lb_status));
        }
        size_t w = std::max(words, (size_t)1 << 20);
        QE_HIP(hipMalloc(&c->lb_status, w * sizeof(uint64_t)));
        QE_HIP(hipMemsetAsync(c->lb_status, 0, w * sizeof(uint64_t), c->stream));
        c->lb_status_words = w;
    }
    c->lb_epoch++;
    if (c->lb_epoch >= (uint32_t)LB_MAX_COUNTERS) {
        // epoch wrap: clear every status word and ticket, restart at 1
        QE_HIP(hipMemsetAsync(c->lb_status, 0, c->lb_status_words * sizeof(uint64_t), c->stream));
        QE_HIP(hipMemsetAsync(c->lb_tickets, 0, LB_MAX_COUNTERS * sizeof(uint32_t), c->stream));
        c->lb_epoch = 1;
    }
    return LBSlot{c->lb_status, c->lb_tickets + c->lb_epoch, c->lb_epoch};
}

// ---------------------------------------------------------------------------------------------
// profiling: HIP events on the ctx stream around each launch (bench.py reads these)
// ---------------------------------------------------------------------------------------------
static hipEvent_t get_event(qe_ctx* c) {
    if (!c->event_pool.empty()) {
        hipEvent_t e = c->event_pool.back();
        c->event_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    QE_HIP(hipEventCreate(&e));
    return e;
}

static void drain_events(qe_ctx* c) {
    if (c->pending.empty()) return;
    QE_HIP(hipStreamSynchronize(c->stream));
    for (auto& p : c->pending) {
        float ms = 0;
        QE_HIP(hipEventElapsedTime(&ms, p.a, p.b));
        KStat& k = c->kstats[p.kernel];
        k.launches++;
        k.ms += ms;
        k.bytes += p.bytes;
        c->event_pool.push_back(p.a);
        c->event_pool.push_back(p.b);
    }
    c->pending.clear();
}

// bytes known only after a launch (its output size) go to that launch's pending record -- only
// if the last one recorded IS that stage (a stage filter may have skipped it)
void add_bytes(qe_ctx* c, const char* stage, double bytes) {
    if (!c->prof || c->pending.empty()) return;
    PendingEvent& p = c->pending.back();
    if (p.kernel >= 0 && (size_t)p.kernel < c->kstats.size() && c->kstats[p.kernel].name == stage) p.bytes += bytes;
}

Timed::Timed(qe_ctx* c_, const char* name, double alg_bytes) : c(c_), bytes(alg_bytes) {
    if (!c->prof || (!c->prof_only.empty() && c->prof_only != name)) return;
    auto it = c->kindex.find(name);
    if (it == c->kindex.end()) {
        k = (int)c->kstats.size();
        c->kindex[name] = k;
        KStat s;
        s.name = name;
        c->kstats.push_back(s);
    } else {
        k = it->second;
    }
    a = get_event(c);
    b = get_event(c);
    QE_HIP(hipEventRecord(a, c->stream));
}

Timed::~Timed() {
    if (!c->prof || k < 0) return;
    if (hipEventRecord(b, c->stream) != hipSuccess) return;
    c->pending.push_back(PendingEvent{k, a, b, bytes});
    if (c->pending.size() > 4096) {
        try {
            drain_events(c);
        } catch (...) {
        }
    }
}

// profiling: a host round trip (the host waits for the GPU) counts as one "launch" of the
// zero-time stage host_round_trip, so bench.py reports round trips per query beside the kernels
static void count_stage(qe_ctx* c, const std::string& name) {
    auto it = c->kindex.find(name);
    int k;
    if (it == c->kindex.end()) {
        k = (int)c->kstats.size();
        c->kindex[name] = k;
        KStat s;
        s.name = name;
        c->kstats.push_back(s);
    } else {
        k = it->second;
    }
    c->kstats[k].launches++;
}

// QE_RT_SITES=1: each round trip also counts under "rt@<file>:<line>" (which calls make them)
static void count_round_trip(qe_ctx* c, const char* file, int line) {
    if (!c->prof) return;
    count_stage(c, "host_round_trip");
    static const bool sites = getenv("QE_RT_SITES") && getenv("QE_RT_SITES")[0] == '1';
    if (sites) {
        const char* b = strrchr(file, '/');
        count_stage(c, std::string("rt@") + (b ? b + 1 : file) + ":" + std::to_string(line));
    }
}

void sync(qe_ctx* c, const char* file, int line) {
    count_round_trip(c, file, line);
    QE_HIP(hipStreamSynchronize(c->stream));
}

// Scalar results the host needs to go on (a list length, a pair count, a sum): one kernel copies
// them from HBM into pinned coherent host memory and then raises a sequence number there (a
// system-scope release: one wave, so its lanes' stores are all ordered before the flag); the host
// spins on that word in its own memory -- no HIP runtime call in the wait loop.  The round-3 wait
// (hipEventQuery spun by up to 8 lane threads at once) took ~22 us less per result than
// hipStreamSynchronize but crashed inside the runtime under rocprofv3's kernel trace with the
// bench's timing events on.  A wait longer than ~2 ms blocks in
// hipStreamSynchronize once (which also surfaces a faulted stream) before the flag is re-read.
// QE_WAIT=event: the round-3 event spin; QE_WAIT=sync: copy + hipStreamSynchronize.
constexpr int RET_WORDS = 512;
__global__ void __launch_bounds__(256) publish_kernel(const uint64_t* __restrict__ d, int n, uint64_t* out,
                                                      uint64_t seq) {
    for (int i = threadIdx.x; i < n; i += 256)
        __hip_atomic_store(&out[1 + i], d[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(&out[0], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

enum { WAIT_FLAG = 0, WAIT_EVENT = 1, WAIT_SYNC = 2 };
static int wait_mode() {
    static const int m = [] {
        const char* s = getenv("QE_WAIT");
        if (const char* o = getenv("QE_SPIN_WAIT"); o && o[0] == '0') return (int)WAIT_SYNC;   // (round-3 knob)
        if (!s) return (int)WAIT_FLAG;
        return !strcmp(s, "event") ? (int)WAIT_EVENT : !strcmp(s, "sync") ? (int)WAIT_SYNC : (int)WAIT_FLAG;
    }();
    return m;
}

static void wait_event(qe_ctx* c) {
    if (!c->wait_ev) QE_HIP(hipEventCreateWithFlags(&c->wait_ev, hipEventDisableTiming));
    QE_HIP(hipEventRecord(c->wait_ev, c->stream));
    hipError_t e;
    while ((e = hipEventQuery(c->wait_ev)) == hipErrorNotReady) {
    }
    QE_HIP(e);
}

// h[0..n) = d[0..n) (device words), the one host round trip of a result
void read_words(qe_ctx* c, const uint64_t* d, uint64_t* h, int n, const char* file, int line) {
    count_round_trip(c, file, line);
    const int mode = wait_mode();
    if (mode != WAIT_FLAG || n > RET_WORDS) {
        QE_HIP(hipMemcpyAsync(c->h_scratch, d, n * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
        if (mode == WAIT_EVENT) wait_event(c);
        else QE_HIP(hipStreamSynchronize(c->stream));
        memcpy(h, c->h_scratch, n * sizeof(uint64_t));
        return;
    }
    if (!c->h_ret) {
        QE_HIP(hipHostMalloc((void**)&c->h_ret, (1 + RET_WORDS) * sizeof(uint64_t),
                             hipHostMallocCoherent | hipHostMallocMapped));
        QE_HIP(hipHostGetDevicePointer((void**)&c->d_ret, c->h_ret, 0));
        __atomic_store_n(&c->h_ret[0], 0ull, __ATOMIC_RELEASE);
        c->ret_seq = 0;
    }
    const uint64_t seq = ++c->ret_seq;
    hipLaunchKernelGGL(publish_kernel, dim3(1), dim3(256), 0, c->stream, d, n, c->d_ret, seq);
    QE_HIP(hipGetLastError());
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spins = 1; __atomic_load_n(&c->h_ret[0], __ATOMIC_ACQUIRE) != seq; spins++) {
        if ((spins & 255) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(2000)) {
            QE_HIP(hipStreamSynchronize(c->stream));   // a long wait: block once (errors surface here)
            if (__atomic_load_n(&c->h_ret[0], __ATOMIC_ACQUIRE) != seq)
                throw Error(QE_EINVAL, "internal: a result's sequence flag never arrived");
            break;
        }
        __builtin_ia32_pause();
    }
    for (int i = 0; i < n; i++) h[i] = __atomic_load_n(&c->h_ret[1 + i], __ATOMIC_RELAXED);
}

uint64_t read_u64(qe_ctx* c, const uint64_t* d, const char* file, int line) {
    uint64_t v;
    read_words(c, d, &v, 1, file, line);
    return v;
}

// ---------------------------------------------------------------------------------------------
// generator: v = splitmix64(((seed<<40)|(rel<<36)|(col<<32)) + row)  
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void __launch_bounds__(256) gen_column_kernel(uint64_t* out, uint64_t rows, uint64_t base,
                                                         uint64_t row_start, int kind, uint64_t mod) {
    uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows; i += stride) {
        uint64_t v = splitmix64(base + row_start + i);
        out[i] = kind == 0 ? v % mod : (v >> 32);
    }
}

// ---- Zipf keys (C5): inverse CDF through a guide table, then a seeded Feistel permutation ----
constexpr int ZG_BITS = 24;                       // guide: 2^24 + 1 entries
constexpr uint64_t ZG_M = 1ull << ZG_BITS;

// guide[j] = #{r : cdf[r] < j / M}: a draw u in [j/M, (j+1)/M) has its rank in [guide[j], guide[j+1]]
__global__ void __launch_bounds__(256) zipf_guide_kernel(const double* __restrict__ cdf, uint64_t d,
                                                         uint64_t* __restrict__ guide) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j > ZG_M) return;
    const double t = (double)j * (1.0 / (double)ZG_M);
    uint64_t lo = 0, hi = d;                      // first r with cdf[r] >= t
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (cdf[mid] < t) lo = mid + 1;
        else hi = mid;
    }
    guide[j] = lo;
}

// 4 rounds on b-bit words (b even), cycle-walked into [0, d): qe/datagen.py feistel_perm
__device__ __forceinline__ uint64_t feistel_perm(uint64_t x, uint64_t d, uint32_t half, uint64_t k0, uint64_t k1,
                                                 uint64_t k2, uint64_t k3) {
    const uint64_t mask = (1ull << half) - 1;
    do {
        uint64_t lo = x & mask, hi = x >> half;
        uint64_t t;
        t = hi ^ (splitmix64(lo + k0) & mask); hi = lo; lo = t;
        t = hi ^ (splitmix64(lo + k1) & mask); hi = lo; lo = t;
        t = hi ^ (splitmix64(lo + k2) & mask); hi = lo; lo = t;
        t = hi ^ (splitmix64(lo + k3) & mask); hi = lo; lo = t;
        x = (hi << half) | lo;
    } while (x >= d);
    return x;
}

// deterministic Zipf CDF: w_r = (r + 1)^-theta summed in a fixed order -- 16 consecutive terms
// per thread, a fixed shuffle tree per wave and block, one thread per 4096-term block prefix --
// so every run on the device builds the same table (a library scan with a decoupled look-back
// adds in a timing-dependent order and changes the low bits run to run)
constexpr int ZC_ITEMS = 16, ZC_B = 256, ZC_CHUNK = ZC_ITEMS * ZC_B;

__device__ __forceinline__ double zipf_w(uint64_t r, double theta) { return pow((double)(r + 1), -theta); }

__device__ __forceinline__ double wave_incl_scan_f64(double v) {
    const int l = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const double o = __shfl_up(v, d, 64);
        if (l >= d) v += o;
    }
    return v;
}

__global__ void __launch_bounds__(ZC_B) zipf_block_sums(uint64_t d, double theta, double* __restrict__ bsum) {
    __shared__ double red[ZC_B / 64];
    const uint64_t i0 = (uint64_t)blockIdx.x * ZC_CHUNK + (uint64_t)threadIdx.x * ZC_ITEMS;
    double s = 0;
    for (int j = 0; j < ZC_ITEMS; j++)
        if (i0 + j < d) s += zipf_w(i0 + j, theta);
    s = wave_incl_scan_f64(s);
    if ((threadIdx.x & 63) == 63) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) bsum[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

__global__ void __launch_bounds__(1) zipf_block_prefix(double* __restrict__ bsum, uint64_t nb) {
    double run = 0;   // serial over <= 2.5e5 block sums: fixed order, ~1 ms at D = 1e9
    for (uint64_t b = 0; b < nb; b++) {
        const double v = bsum[b];
        bsum[b] = run;
        run += v;
    }
}

__global__ void __launch_bounds__(ZC_B) zipf_block_scan(uint64_t d, double theta, const double* __restrict__ bpre,
                                                        double* __restrict__ cdf) {
    __shared__ double red[ZC_B / 64];
    const uint64_t i0 = (uint64_t)blockIdx.x * ZC_CHUNK + (uint64_t)threadIdx.x * ZC_ITEMS;
    double w[ZC_ITEMS], s = 0;
    for (int j = 0; j < ZC_ITEMS; j++) {
        w[j] = i0 + j < d ? zipf_w(i0 + j, theta) : 0.0;
        s += w[j];
    }
    const double inc = wave_incl_scan_f64(s);
    if ((threadIdx.x & 63) == 63) red[threadIdx.x >> 6] = inc;
    __syncthreads();
    double run = bpre[blockIdx.x];
    for (int q = 0; q < (int)(threadIdx.x >> 6); q++) run += red[q];
    run += inc - s;
    for (int j = 0; j < ZC_ITEMS; j++) {
        run += w[j];
        if (i0 + j < d) cdf[i0 + j] = run;
    }
}

// cdf /= total (total: a copy of the last entry, which becomes exactly 1.0)
__global__ void __launch_bounds__(256) zipf_normalise(uint64_t d, double* __restrict__ cdf,
                                                      const double* __restrict__ total) {
    const double last = *total;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < d; i += stride) cdf[i] = cdf[i] / last;
}

__global__ void __launch_bounds__(256) gen_zipf_kernel(uint64_t* __restrict__ out, uint64_t rows, uint64_t base,
                                                       uint64_t row_start, const double* __restrict__ cdf,
                                                       const uint64_t* __restrict__ guide, uint64_t d, uint32_t half,
                                                       uint64_t k0, uint64_t k1, uint64_t k2, uint64_t k3) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows; i += stride) {
        const uint64_t v = splitmix64(base + row_start + i);
        const double u = (double)(v >> 11) * (1.0 / 9007199254740992.0);
        const uint64_t j = (uint64_t)(u * (double)ZG_M);          // exact: M is a power of two
        uint64_t lo = guide[j], hi = guide[j + 1];                  // rank in [lo, hi]
        while (lo < hi) {                                           // first r >= lo with cdf[r] > u
            const uint64_t mid = (lo + hi) >> 1;
            if (cdf[mid] <= u) lo = mid + 1;
            else hi = mid;
        }
        const uint64_t rank = lo < d ? lo : d - 1;
        out[i] = feistel_perm(rank, d, half, k0, k1, k2, k3);
    }
}

}  // namespace qe

using namespace qe;

namespace qe {
__global__ void __launch_bounds__(256) narrow_kernel(const uint64_t* __restrict__ in, uint64_t n,
                                                     uint32_t* __restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) out[i] = (uint32_t)in[i];
}
}  // namespace qe

static void free_relation(Relation& r) {
    if (!r.owned) return;
    for (auto* p : r.cols) (void)hipFree(p);
    for (auto* p : r.cols32)
        if (p) (void)hipFree(p);
}

// column statistics: OR / AND of every column, one read at load time (zone-map style metadata
// that lets the radix sort plan its passes without a reduction pass per query); and a u32 copy of
// every column whose values fit 32 bits -- the relation's second layout in HBM, the one the
// sorts' first passes read (QE_NARROW=0: none; a copy that does not fit in memory is skipped)
static void column_stats(qe_ctx* c, Relation& r) {
    r.kor.resize(r.cols.size());
    r.kand.resize(r.cols.size());
    for (size_t j = 0; j < r.cols.size(); j++) {
        uint64_t b[2];
        key_bits_u64(c, r.cols[j], r.rows, b);
        r.kor[j] = b[0];
        r.kand[j] = b[1];
    }
    const char* e = getenv("QE_NARROW");
    r.cols32.assign(r.cols.size(), nullptr);
    if (e && e[0] == '0') return;
    try {
        for (size_t j = 0; j < r.cols.size(); j++) {
            if ((r.kor[j] >> 32) || !r.rows) continue;
            uint32_t* d = nullptr;
            if (hipMalloc(&d, r.rows * sizeof(uint32_t) + DALLOC_SLACK) != hipSuccess) {   // (slack: as dalloc's)
                // best effort: a relation near the memory limit loads without its u32 copies
                // (every reader of cols32 takes the u64 column when the copy is null)
                (void)hipGetLastError();
                continue;
            }
            r.cols32[j] = d;
            hipLaunchKernelGGL(narrow_kernel, dim3(grid_for(r.rows, 256 * 8, 16384)), dim3(256), 0, c->stream,
                               r.cols[j], r.rows, d);
            QE_HIP(hipGetLastError());
        }
        QE_HIP(hipStreamSynchronize(c->stream));
    } catch (...) {   // (the caller's guard frees the u64 columns)
        for (auto*& p : r.cols32)
            if (p) (void)hipFree(p), p = nullptr;
        throw;
    }
}

// Host -> HBM copy of a pageable buffer (an mmap'd relation file, a numpy column): a ring of
// pinned 32 MiB slots.  Each slot is filled by several host threads (one thread's memcpy is
// ~10 GB/s, well below a PCIe5 x16 link) and copied with hipMemcpyAsync while the next slot
// fills; a slot is refilled once its previous copy has completed (event).  (hipMemcpy from
// pageable memory stages through the runtime's own small buffers, one chunk at a time.)
static void h2d_staged(qe_ctx* c, void* dst, const void* src, size_t bytes) {
    constexpr size_t SLOT = 32ull << 20;
    if (!c->h_stage[0]) {
        for (int k = 0; k < qe_ctx::STAGE_SLOTS; k++) {
            QE_HIP(hipHostMalloc(&c->h_stage[k], SLOT, hipHostMallocDefault));
            QE_HIP(hipEventCreateWithFlags(&c->stage_ev[k], hipEventDisableTiming));
        }
        c->stage_bytes = SLOT;
    }
    unsigned nth = std::thread::hardware_concurrency();
    nth = nth < 2 ? 1 : (nth > 8 ? 8 : nth);
    if (const char* e = getenv("QE_LOAD_THREADS")) nth = (unsigned)std::max(1, atoi(e));
    int k = 0;
    for (size_t off = 0; off < bytes; off += SLOT, k = (k + 1) % qe_ctx::STAGE_SLOTS) {
        const size_t len = std::min(SLOT, bytes - off);
        QE_HIP(hipEventSynchronize(c->stage_ev[k]));   // the slot's previous copy is done
        char* stage = static_cast<char*>(c->h_stage[k]);
        const char* from = static_cast<const char*>(src) + off;
        if (nth == 1 || len < (1u << 20)) {
            memcpy(stage, from, len);
        } else {
            std::vector<std::thread> th;
            const size_t per = (len / nth + 4095) & ~(size_t)4095;
            for (unsigned t = 0; t < nth; t++) {
                const size_t a = t * per;
                if (a >= len) break;
                const size_t b = std::min(len, a + per);
                th.emplace_back([=] { memcpy(stage + a, from + a, b - a); });
            }
            for (auto& x : th) x.join();
        }
        QE_HIP(hipMemcpyAsync(static_cast<char*>(dst) + off, stage, len, hipMemcpyHostToDevice, c->stream));
        QE_HIP(hipEventRecord(c->stage_ev[k], c->stream));
    }
}

// =============================================================================================
// C ABI: lifecycle, relations, buffers, profiling
// =============================================================================================
extern "C" {

int qe_abi_version(void) { return QE_ABI_VERSION; }

qe_ctx* qe_init(int device) {
    qe_ctx* c = new qe_ctx();
    c->device = device;
    try {
        QE_HIP(hipSetDevice(device));
        QE_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        QE_HIP(hipMalloc(&c->lb_tickets, LB_MAX_COUNTERS * sizeof(uint32_t)));
        QE_HIP(hipMemsetAsync(c->lb_tickets, 0, LB_MAX_COUNTERS * sizeof(uint32_t), c->stream));
        QE_HIP(hipMalloc(&c->d_scratch, 64 * sizeof(uint64_t)));
        QE_HIP(hipHostMalloc((void**)&c->h_scratch, 64 * sizeof(uint64_t), hipHostMallocDefault));
        QE_HIP(hipStreamSynchronize(c->stream));
        if (const char* e = getenv("QE_MAT_LIMIT")) c->mat_limit = strtoull(e, nullptr, 0);
    } catch (const Error& e) {
        fprintf(stderr, "qe_init(%d): %s\n", device, e.what());
        delete c;
        return nullptr;
    }
    return c;
}

void qe_fini(qe_ctx* c) {
    if (!c) return;
    for (qe_ctx* w : c->workers) qe_fini(w);   // (they borrow this ctx's relations)
    c->workers.clear();
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    if (c->side.stream) (void)hipStreamSynchronize(c->side.stream);
    for (auto& r : c->rels) free_relation(r);
    for (auto& kv : c->free_blocks) hfree(c, kv.second);
    for (auto& kv : c->live) hfree(c, kv.first);
    for (auto& p : c->pending) {
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    for (auto e : c->event_pool) (void)hipEventDestroy(e);
    if (c->lb_status) (void)hipFree(c->lb_status);
    if (c->lb_tickets) (void)hipFree(c->lb_tickets);
    if (c->d_scratch) (void)hipFree(c->d_scratch);
    if (c->d_zhist) (void)hipFree(c->d_zhist);
    if (c->h_scratch) (void)hipHostFree(c->h_scratch);
    if (c->h_ret) (void)hipHostFree(c->h_ret);
    if (c->wait_ev) (void)hipEventDestroy(c->wait_ev);
    {   // the side stream's state (never swapped in here: SideFork restores the main one)
        StreamState& s = c->side;
        if (s.stream) (void)hipStreamSynchronize(s.stream);
        if (s.lb_status) (void)hipFree(s.lb_status);
        if (s.lb_tickets) (void)hipFree(s.lb_tickets);
        if (s.d_scratch) (void)hipFree(s.d_scratch);
        if (s.d_zhist) (void)hipFree(s.d_zhist);
        if (s.h_scratch) (void)hipHostFree(s.h_scratch);
        if (s.h_ret) (void)hipHostFree(s.h_ret);
        if (s.wait_ev) (void)hipEventDestroy(s.wait_ev);
        if (s.stream) (void)hipStreamDestroy(s.stream);
        for (auto e : c->fork_ev)
            if (e) (void)hipEventDestroy(e);
    }
    for (int k = 0; k < qe_ctx::STAGE_SLOTS; k++) {
        if (c->h_stage[k]) (void)hipHostFree(c->h_stage[k]);
        if (c->stage_ev[k]) (void)hipEventDestroy(c->stage_ev[k]);
    }
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* qe_last_error(qe_ctx* c) { return c ? c->err.c_str() : "null context"; }

int qe_device_name(qe_ctx* c, char* out, size_t cap) {
    QE_API_BEGIN(c)
    hipDeviceProp_t p;
    QE_HIP(hipGetDeviceProperties(&p, c->device));
    snprintf(out, cap, "%s (%s, %d CUs)", p.name, p.gcnArchName, p.multiProcessorCount);
    return 0;
    QE_API_END(c)
}

int qe_sync(qe_ctx* c) {
    QE_API_BEGIN(c)
    sync(c);
    return 0;
    QE_API_END(c)
}

/* frees a relation's columns unless the relation was stored (a failed load or generate must not
 * leak the columns it already allocated) */
struct ColsGuard {
    std::vector<uint64_t*>& cols;
    bool keep = false;
    explicit ColsGuard(std::vector<uint64_t*>& v) : cols(v) {}
    ~ColsGuard() {
        if (keep) return;
        for (uint64_t* d : cols) (void)hipFree(d);
        cols.clear();
    }
};

int qe_load_relation(qe_ctx* c, uint64_t rows, uint64_t ncols, const uint64_t* const* host_cols) {
    QE_API_BEGIN(c)
    if (rows >= 0xFFFFFFFFull) throw Error(QE_EINVAL, "relation too large for uint32 rowids");
    Relation r;
    r.rows = rows;
    ColsGuard guard(r.cols);
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t j = 0; j < ncols; j++) {
        uint64_t* d = nullptr;
        QE_HIP(hipMalloc(&d, std::max<uint64_t>(rows, 1) * sizeof(uint64_t) + DALLOC_SLACK));   // (slack: as dalloc's)
        r.cols.push_back(d);
        if (!rows) continue;
        if (getenv("QE_LOAD_DIRECT"))   // A/B only: the runtime's own pageable copy
            QE_HIP(hipMemcpyAsync(d, host_cols[j], rows * sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
        else
            h2d_staged(c, d, host_cols[j], rows * sizeof(uint64_t));
    }
    QE_HIP(hipStreamSynchronize(c->stream));
    column_stats(c, r);   // (its OR/AND read and u32 copies are part of the load: timed with it)
    c->load_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    c->load_bytes += (double)rows * ncols * sizeof(uint64_t);
    guard.keep = true;
    c->rels.push_back(std::move(r));
    return (int)c->rels.size() - 1;
    QE_API_END(c)
}

int qe_gen_relation(qe_ctx* c, uint64_t rows, uint64_t ncols, const int* kinds, const uint64_t* mods,
                    uint64_t seed, uint32_t gen_rel, uint64_t row_start) {
    QE_API_BEGIN(c)
    if (rows >= 0xFFFFFFFFull) throw Error(QE_EINVAL, "relation too large for uint32 rowids");
    for (uint64_t j = 0; j < ncols; j++) {      /* every column checked before anything is allocated */
        if (kinds[j] == 0 && mods[j] == 0) throw Error(QE_EINVAL, "mod 0");
        if (kinds[j] == 2 && (!c->zipf_cdf || mods[j] != c->zipf_domain))
            throw Error(QE_EINVAL, "no Zipf table for this domain");
        if (kinds[j] < 0 || kinds[j] > 2) throw Error(QE_EINVAL, "unknown column kind");
    }
    Relation r;
    r.rows = rows;
    ColsGuard guard(r.cols);
    for (uint64_t j = 0; j < ncols; j++) {
        uint64_t* d = nullptr;
        QE_HIP(hipMalloc(&d, std::max<uint64_t>(rows, 1) * sizeof(uint64_t) + DALLOC_SLACK));   // (slack: as dalloc's)
        r.cols.push_back(d);
        uint64_t base = (seed << 40) | ((uint64_t)gen_rel << 36) | ((uint64_t)j << 32);
        if (kinds[j] == 2) {
            uint32_t b = 2;
            while (b < 64 && ((c->zipf_domain - 1) >> b) != 0) b++;
            b += b & 1;
            uint64_t k[4];
            for (int r = 0; r < 4; r++) k[r] = (c->zipf_perm_seed << 40) | (15ull << 36) | ((uint64_t)r << 32);
            if (rows)
                hipLaunchKernelGGL(gen_zipf_kernel, dim3(grid_for(rows, 256 * 8, 8192)), dim3(256), 0, c->stream, d,
                                   rows, base, row_start, c->zipf_cdf, c->zipf_guide, c->zipf_domain, b / 2, k[0],
                                   k[1], k[2], k[3]);
        } else if (rows) {
            hipLaunchKernelGGL(gen_column_kernel, dim3(grid_for(rows, 256 * 8, 8192)), dim3(256), 0, c->stream, d,
                               rows, base, row_start, kinds[j], mods[j]);
        }
        QE_HIP(hipGetLastError());
    }
    QE_HIP(hipStreamSynchronize(c->stream));
    column_stats(c, r);
    guard.keep = true;
    c->rels.push_back(std::move(r));
    return (int)c->rels.size() - 1;
    QE_API_END(c)
}

int qe_last_result_rows(qe_ctx* c, uint64_t* rows) {
    if (!c) return QE_EINVAL;
    *rows = c->last_result_rows;
    return 0;
}

int qe_set_last_result_rows(qe_ctx* c, uint64_t rows) {
    if (!c) return QE_EINVAL;
    c->last_result_rows = rows;
    return 0;
}

int qe_set_zipf(qe_ctx* c, uint64_t domain, double theta, uint64_t perm_seed) {
    QE_API_BEGIN(c)
    if (domain == 0) throw Error(QE_EINVAL, "empty Zipf domain");
    double* cdf = dalloc_t<double>(c, domain);
    const uint64_t nb = (domain + ZC_CHUNK - 1) / ZC_CHUNK;
    double* bsum = dalloc_t<double>(c, nb + 1);
    hipLaunchKernelGGL(zipf_block_sums, dim3((unsigned)nb), dim3(ZC_B), 0, c->stream, domain, theta, bsum);
    QE_HIP(hipGetLastError());
    hipLaunchKernelGGL(zipf_block_prefix, dim3(1), dim3(1), 0, c->stream, bsum, nb);
    QE_HIP(hipGetLastError());
    hipLaunchKernelGGL(zipf_block_scan, dim3((unsigned)nb), dim3(ZC_B), 0, c->stream, domain, theta, bsum, cdf);
    QE_HIP(hipGetLastError());
    QE_HIP(hipMemcpyAsync(bsum + nb, cdf + domain - 1, 8, hipMemcpyDeviceToDevice, c->stream));
    hipLaunchKernelGGL(zipf_normalise, dim3(grid_for(domain, 256 * 8, 8192)), dim3(256), 0, c->stream, domain, cdf,
                       bsum + nb);
    QE_HIP(hipGetLastError());
    const int rc = qe_set_zipf_table(c, cdf, domain, perm_seed);
    dfree(c, bsum);
    if (rc != 0) {
        dfree(c, cdf);
        return rc;
    }
    c->zipf_owned = cdf;
    return 0;
    QE_API_END(c)
}

int qe_set_zipf_table(qe_ctx* c, const double* d_cdf, uint64_t domain, uint64_t perm_seed) {
    QE_API_BEGIN(c)
    if (c->zipf_guide) dfree(c, c->zipf_guide);
    if (c->zipf_owned && c->zipf_owned != d_cdf) dfree(c, c->zipf_owned);
    c->zipf_owned = nullptr;
    c->zipf_guide = nullptr;
    c->zipf_cdf = nullptr;
    c->zipf_domain = 0;
    if (!d_cdf) return 0;
    if (domain == 0) throw Error(QE_EINVAL, "empty Zipf domain");
    c->zipf_guide = dalloc_t<uint64_t>(c, ZG_M + 1);
    hipLaunchKernelGGL(zipf_guide_kernel, dim3((unsigned)((ZG_M + 1 + 255) / 256)), dim3(256), 0, c->stream, d_cdf,
                       domain, c->zipf_guide);
    QE_HIP(hipGetLastError());
    c->zipf_cdf = d_cdf;
    c->zipf_domain = domain;
    c->zipf_perm_seed = perm_seed;
    sync(c);
    return 0;
    QE_API_END(c)
}

int qe_relation_count(qe_ctx* c) { return c ? (int)c->rels.size() : QE_EINVAL; }

int qe_relation_column(qe_ctx* c, int rel, int col, qe_col* out) {
    if (!c || rel < 0 || rel >= (int)c->rels.size() || col < 0 || col >= (int)c->rels[rel].cols.size())
        return QE_EINVAL;
    out->d = c->rels[rel].cols[col];
    out->n = c->rels[rel].rows;
    return 0;
}

int qe_relation_column_bits(qe_ctx* c, int rel, int col, uint64_t* kor, uint64_t* kand) {
    if (!c || rel < 0 || rel >= (int)c->rels.size() || col < 0 || col >= (int)c->rels[rel].cols.size())
        return QE_EINVAL;
    *kor = c->rels[rel].kor[col];
    *kand = c->rels[rel].kand[col];
    return 0;
}

int qe_relation_rows(qe_ctx* c, int rel, uint64_t* rows) {
    if (!c || rel < 0 || rel >= (int)c->rels.size()) return QE_EINVAL;
    *rows = c->rels[rel].rows;
    return 0;
}

int qe_drop_relations(qe_ctx* c) {
    QE_API_BEGIN(c)
    for (qe_ctx* w : c->workers) {             // workers may still read them
        sync(w);
        w->rels.clear();
        qe::drop_partitions(w);
    }
    qe::drop_partitions(c);
    sync(c);
    for (auto& r : c->rels) free_relation(r);
    c->rels.clear();
    return 0;
    QE_API_END(c)
}

int qe_workers(qe_ctx* c, int n, qe_ctx** out) {
    QE_API_BEGIN(c)
    if (n < 1 || n > 16) throw Error(QE_EINVAL, "1..16 workers");
    while ((int)c->workers.size() < n) {
        qe_ctx* w = qe_init(c->device);
        if (!w) throw Error(QE_EHIP, "worker context");
        c->workers.push_back(w);
    }
    sync(c);                                   // the relations are complete before a worker reads them
    for (int i = 0; i < n; i++) {
        qe_ctx* w = c->workers[i];
        w->rels.clear();
        for (const auto& r : c->rels) {
            Relation b = r;
            b.owned = false;
            w->rels.push_back(b);
        }
        w->mat_limit = c->mat_limit;
        w->prof = c->prof;
        w->scache = c->scache;
        out[i] = w;
    }
    return 0;
    QE_API_END(c)
}

int qe_bind_thread(qe_ctx* c) {
    if (!c) return QE_EINVAL;
    return hipSetDevice(c->device) == hipSuccess ? 0 : QE_EHIP;
}

void qe_free_host(void* p) { free(p); }

int qe_list_alloc(qe_ctx* c, uint64_t n, qe_list* out) {
    QE_API_BEGIN(c)
    out->d = dalloc_t<uint32_t>(c, std::max<uint64_t>(n, 1));
    out->n = 0;
    out->cap = n;
    out->flags = 0;
    return 0;
    QE_API_END(c)
}

int qe_list_from_host(qe_ctx* c, const uint32_t* h, uint64_t n, uint32_t flags, qe_list* out) {
    QE_API_BEGIN(c)
    out->d = dalloc_t<uint32_t>(c, std::max<uint64_t>(n, 1));
    if (n) QE_HIP(hipMemcpyAsync(out->d, h, n * 4, hipMemcpyHostToDevice, c->stream));
    QE_HIP(hipStreamSynchronize(c->stream));
    out->n = n;
    out->cap = n;
    out->flags = flags;
    return 0;
    QE_API_END(c)
}

int qe_list_to_host(qe_ctx* c, const qe_list* l, uint32_t* h) {
    QE_API_BEGIN(c)
    if (l->n) QE_HIP(hipMemcpyAsync(h, l->d, l->n * 4, hipMemcpyDeviceToHost, c->stream));
    QE_HIP(hipStreamSynchronize(c->stream));
    return 0;
    QE_API_END(c)
}

void qe_list_free(qe_ctx* c, qe_list* l) {
    if (!c || !l) return;
    dfree(c, l->d);
    l->d = nullptr;
    l->n = l->cap = 0;
}

int qe_pairs_from_host(qe_ctx* c, const uint64_t* key, const uint32_t* val, uint64_t n, qe_pairs* out) {
    QE_API_BEGIN(c)
    out->key = dalloc_t<uint64_t>(c, std::max<uint64_t>(n, 1));
    out->val = dalloc_t<uint32_t>(c, std::max<uint64_t>(n, 1));
    if (n) {
        QE_HIP(hipMemcpyAsync(out->key, key, n * 8, hipMemcpyHostToDevice, c->stream));
        QE_HIP(hipMemcpyAsync(out->val, val, n * 4, hipMemcpyHostToDevice, c->stream));
    }
    QE_HIP(hipStreamSynchronize(c->stream));
    out->match = nullptr;
    out->n = n;
    out->kor = out->kand = 0;
    out->flags = 0;
    out->owns = 3;
    return 0;
    QE_API_END(c)
}

int qe_pairs_to_host(qe_ctx* c, const qe_pairs* p, uint64_t* key, uint32_t* val) {
    QE_API_BEGIN(c)
    pairs_need_keys(c, p);
    if (p->n) {
        if (key) QE_HIP(hipMemcpyAsync(key, p->key, p->n * 8, hipMemcpyDeviceToHost, c->stream));
        if (val) {
            if (p->val) {
                QE_HIP(hipMemcpyAsync(val, p->val, p->n * 4, hipMemcpyDeviceToHost, c->stream));
            } else {
                QE_HIP(hipStreamSynchronize(c->stream));
                for (uint64_t i = 0; i < p->n; i++) val[i] = (uint32_t)i;
            }
        }
    }
    QE_HIP(hipStreamSynchronize(c->stream));
    return 0;
    QE_API_END(c)
}

void qe_pairs_free(qe_ctx* c, qe_pairs* p) {
    if (!c || !p) return;
    // (pairs that only borrow their key buffer leave its u32 keys, PreHist::k32, to its owner:
    // a join that gives its inputs back is followed by another sort of the same buffer)
    pairs_drop_deferred(c, p, !(p->owns & 1));
    if (p->owns & 1) dfree(c, p->key);
    if (p->owns & 2) dfree(c, p->val);
    if (p->owns & 4) dfree(c, p->match);
    p->match = nullptr;
    p->key = nullptr;
    p->val = nullptr;
    p->n = 0;
    p->owns = 0;
}

void qe_counts_free(qe_ctx* c, uint32_t* d) {
    if (c) dfree(c, d);
}

int qe_counts_to_host(qe_ctx* c, const uint32_t* d, uint64_t n, uint32_t* h) {
    QE_API_BEGIN(c)
    if (n) QE_HIP(hipMemcpyAsync(h, d, n * 4, hipMemcpyDeviceToHost, c->stream));
    QE_HIP(hipStreamSynchronize(c->stream));
    return 0;
    QE_API_END(c)
}

int qe_load_stats(qe_ctx* c, double* seconds, double* bytes) {
    QE_API_BEGIN(c)
    *seconds = c->load_s;
    *bytes = c->load_bytes;
    return 0;
    QE_API_END(c)
}

int qe_mem_stats(qe_ctx* c, uint64_t* in_use, uint64_t* cached) {
    if (!c) return QE_EINVAL;
    *in_use = c->in_use;
    *cached = c->cached;
    return 0;
}

int qe_mem_trim(qe_ctx* c) {
    QE_API_BEGIN(c)
    sync(c);
    for (auto& kv : c->free_blocks) hfree(c, kv.second);
    c->free_blocks.clear();
    c->cached = 0;
    return 0;
    QE_API_END(c)
}

// profiling covers a ctx and its worker contexts (qe_run_queries_parallel's lanes): statistics
// of kernels with one name are summed (the lanes' durations overlap in time)
int qe_set_profiling(qe_ctx* c, int on) {
    QE_API_BEGIN(c)
    drain_events(c);
    c->prof = on != 0;
    for (qe_ctx* w : c->workers) {
        drain_events(w);
        w->prof = c->prof;
    }
    return 0;
    QE_API_END(c)
}


int qe_set_profiling_only(qe_ctx* c, const char* stage) {
    QE_API_BEGIN(c)
    drain_events(c);
    c->prof_only = stage ? stage : "";
    for (qe_ctx* w : c->workers) {
        drain_events(w);
        w->prof_only = c->prof_only;
    }
    return 0;
    QE_API_END(c)
}

int qe_reset_stats(qe_ctx* c) {
    QE_API_BEGIN(c)
    auto reset = [](qe_ctx* x) {
        drain_events(x);
        for (auto& k : x->kstats) {
            k.launches = 0;
            k.ms = 0;
            k.bytes = 0;
        }
    };
    reset(c);
    for (qe_ctx* w : c->workers) reset(w);
    return 0;
    QE_API_END(c)
}

int qe_kernel_stats(qe_ctx* c, qe_kstat* out, int max) {
    QE_API_BEGIN(c)
    std::vector<KStat> all;
    auto add = [&](qe_ctx* x) {
        drain_events(x);
        for (auto& k : x->kstats) {
            auto it = std::find_if(all.begin(), all.end(), [&](const KStat& a) { return a.name == k.name; });
            if (it == all.end()) {
                all.push_back(k);
            } else {
                it->launches += k.launches;
                it->ms += k.ms;
                it->bytes += k.bytes;
            }
        }
    };
    add(c);
    for (qe_ctx* w : c->workers) add(w);
    int n = 0;
    for (auto& k : all) {
        if (n < max && out) {
            memset(&out[n], 0, sizeof(qe_kstat));
            strncpy(out[n].name, k.name.c_str(), sizeof(out[n].name) - 1);
            out[n].launches = k.launches;
            out[n].total_ms = k.ms;
            out[n].alg_bytes = k.bytes;
        }
        n++;
    }
    return n;
    QE_API_END(c)
}

}  // extern "C"
