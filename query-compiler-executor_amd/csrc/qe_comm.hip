// qe_comm.hip -- multi-GPU half of the C ABI: an RCCL communicator per
// ctx (one process per GPU, xGMI), the key exchange and the all-reduce, and the device engine that
// runs the partitioned plan of include/qe_plan.h (host/qe_plan.c) on libqe's primitives.
//
// The reference has no multi-GPU path; its seam is main/queries_main.c:37 -> execute_queries
// (src/utilities.c:289-300).  qe_run_queries_dist replaces that seam on N ranks: every rank holds
// the relations, queries in the relational domain run partitioned by join key, the others run on
// the faithful executor on rank 0 (qe_exec_query) -- the printed bytes are the reference's either way.
#include <rccl/rccl.h>

#include <unistd.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/qe_plan.h"
#include "../host/qe_query.h"
#include "qe_device.h"
#include "qe_internal.h"

namespace qe {
// The in-process transport (qe_comm_init_local): the ranks are host threads of one process, each
// driving its own ctx -- on a one-GPU box, worker contexts of one device (RCCL refuses two ranks on
// one device).  It replaces exactly the communicator's three RCCL operations: the all-to-all of
// the per-destination counts, the grouped send/recv of the partitioned segments (here: each
// receiver pulls its segment from every sender's partitioned buffer with a device-to-device copy)
// and the all-reduce (host sums).  Partitioning, offsets, the plan and every kernel are the
// production code.  Two barriers per operation: the second keeps a sender's posted buffers alive
// and its posted numbers unchanged until every peer has read them.
struct LocalGroup {
    int n = 0, refs = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    bool broken = false;
    double timeout_s = 600;
    std::vector<std::array<uint64_t, 64>> red, cnt;
    std::vector<const void*> keys;   // each rank's partitioned keys (u64, or u32: Ticket::k32)
    std::vector<std::vector<const uint32_t*>> cols;
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (broken) throw Error(QE_EHIP, "local transport: the group is broken (a peer rank failed)");
        const uint64_t g = gen;
        if (++arrived == n) {
            arrived = 0;
            gen++;
            cv.notify_all();
            return;
        }
        // a peer that never arrives (it failed outside the transport) must not hang the others
        if (!cv.wait_for(lk, std::chrono::duration<double>(timeout_s), [&] { return gen != g || broken; }) || broken) {
            broken = true;
            cv.notify_all();
            throw Error(QE_EHIP, "local transport: a peer rank did not reach the exchange (timeout or failure)");
        }
    }
    void fail() {
        std::lock_guard<std::mutex> lk(mu);
        broken = true;
        cv.notify_all();
    }
};
}  // namespace qe

struct qe_comm {
    ncclComm_t comm = nullptr;
    qe::LocalGroup* local = nullptr;  // in-process transport instead of RCCL (qe_comm_init_local)
    int nranks = 1, rank = 0;
    hipStream_t stream = nullptr;     // exchanges run here, overlapped with the ctx stream's work
    uint64_t* d_red = nullptr;        // all-reduce staging (64 words)
    uint64_t* h_red = nullptr;        // pinned mirror
    uint64_t exchanges = 0, bytes_sent = 0;
};

namespace qe {
namespace {

// a select column's values in a list's order, as u32 (the column's values are below 2^32)
__global__ void __launch_bounds__(256) gather_u32_kernel(const uint64_t* __restrict__ col,
                                                         const uint32_t* __restrict__ rows, uint64_t n,
                                                         uint32_t* __restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * 256 * 4;
    for (uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += stride) {
        if (i + 3 < n) {
            const uint4 r = *reinterpret_cast<const uint4*>(rows + i);
            uint4 v;
            v.x = (uint32_t)col[r.x];
            v.y = (uint32_t)col[r.y];
            v.z = (uint32_t)col[r.z];
            v.w = (uint32_t)col[r.w];
            *reinterpret_cast<uint4*>(out + i) = v;
        } else {
            for (uint64_t k = i; k < n; k++) out[k] = (uint32_t)col[rows[k]];
        }
    }
}

// keys = a list of carried key values, widened (the plain form of widen_with_hist)
__global__ void __launch_bounds__(256) widen_u32_kernel(const uint32_t* __restrict__ v, uint64_t n,
                                                        uint64_t* __restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) out[i] = v[i];
}

// sum of a list's own u32 values mod 2^64 (a binding that carries its select's values)
__global__ void __launch_bounds__(256) sum_u32_kernel(const uint32_t* __restrict__ v, uint64_t n,
                                                      unsigned long long* __restrict__ out) {
    uint64_t t = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 256 * 4;
    for (uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += stride) {
        if (i + 3 < n) {
            const uint4 a = *reinterpret_cast<const uint4*>(v + i);
            t += (uint64_t)a.x + a.y + a.z + a.w;
        } else {
            for (uint64_t k = i; k < n; k++) t += v[k];
        }
    }
    t = wave_sum_u64(t);
    __shared__ uint64_t red[4];
    if (lane_id() == 0) red[wave_id()] = t;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(out, (unsigned long long)(red[0] + red[1] + red[2] + red[3]));
}

#define QE_NCCL(call)                                                                                  \
    do {                                                                                               \
        ncclResult_t r_ = (call);                                                                      \
        if (r_ != ncclSuccess) throw ::qe::Error(QE_EHIP, std::string(#call) + ": " + ncclGetErrorString(r_)); \
    } while (0)

// ---- the device engine: handles are heap objects -------------------------------------------------
struct Obj {
    virtual ~Obj() {}
};

// a device array: rowids (u32) or keys (u64)
struct DArr : Obj {
    qe_ctx* c = nullptr;
    void* d = nullptr;
    uint64_t n = 0;
    bool u64 = false, owned = true;
    bool bits = false;
    uint64_t kor = 0, kand = 0;
    // a fused scan's survivors' values of (vrel, vcol) as u32, kept for a later `values` request
    uint32_t* vcache = nullptr;
    uint32_t vrel = 0, vcol = 0;
    // ... and of (krel, kcol), the binding's join key column, for its key side (e_keys): no gather
    uint32_t* kcache = nullptr;
    uint32_t krel = 0, kcol = 0;
    bool colview = false;   // a base column (e_column): d is the column, n its rows
    ~DArr() override {
        if (vcache) dfree(c, vcache);
        if (kcache) dfree(c, kcache);
        if (owned && d) {
            qe_pairs p{};
            p.key = static_cast<uint64_t*>(d);   // drops a gathered histogram kept for this key buffer
            if (u64) pairs_drop_deferred(c, &p);
            dfree(c, d);
        }
    }
};

struct Ticket : Obj {
    DArr* keys = nullptr;
    void* keys32 = nullptr;           // the received keys as u32 (k32 exchange), widened at finish
    std::vector<DArr*> cols;
    std::vector<void*> send;          // partitioned send buffers, freed once the exchange is done
    hipEvent_t done = nullptr;
};

struct Eng {
    qe_ctx* c;
    qe_comm* comm;
    int world, rank;
    uint64_t refused = 0;
};

inline Eng* E(void* u) { return static_cast<Eng*>(u); }
inline DArr* A(qe_h h) { return reinterpret_cast<DArr*>(h); }
inline qe_h H(Obj* o) { return reinterpret_cast<qe_h>(o); }

DArr* new_arr(qe_ctx* c, void* d, uint64_t n, bool u64, bool owned = true) {
    DArr* a = new DArr;
    a->c = c;
    a->d = d;
    a->n = n;
    a->u64 = u64;
    a->owned = owned;
    return a;
}

qe_list as_list(const DArr* a) {
    qe_list l{};
    l.d = static_cast<uint32_t*>(a->d);
    l.n = a->n;
    l.cap = a->n;
    return l;
}

// a rank that fails outside the plan's agreed outcomes (ETOOBIG and ENOTSUP are all-reduced by the
// plan) will not reach its peers' next collective: an in-process group is told so at once
inline void peer_failed(Eng* e, int code) {
    if (code != QE_ETOOBIG && code != QE_ENOTSUP && e->comm && e->comm->local) e->comm->local->fail();
}

template <class F>
int guard(Eng* e, F f) {
    try {
        f();
        return 0;
    } catch (const Error& x) {
        e->c->err = x.what();
        peer_failed(e, x.code);
        return x.code;
    } catch (const std::exception& x) {
        e->c->err = x.what();
        peer_failed(e, QE_EINVAL);
        return QE_EINVAL;
    }
}

void ck(int rc, qe_ctx* c) {
    if (rc != 0) throw Error(rc, c->err);
}

int e_rel_count(void* u, uint32_t* n) {
    *n = (uint32_t)E(u)->c->rels.size();
    return 0;
}

int e_rel_shape(void* u, uint32_t rel, uint64_t* rows, uint32_t* ncols) {
    qe_ctx* c = E(u)->c;
    if (rel >= c->rels.size()) return QE_EINVAL;
    *rows = c->rels[rel].rows;
    *ncols = (uint32_t)c->rels[rel].cols.size();
    return 0;
}

qe_col column(qe_ctx* c, uint32_t rel, uint32_t col) {
    qe_col q;
    ck(qe_relation_column(c, (int)rel, (int)col, &q), c);
    return q;
}

// the plan's scans: its lists feed only order-free consumers (key gathers before a sort, the
// bucket join, sums), so they come from the unordered wave-tile scan (qe_scan.hip)
int e_scan(void* u, uint32_t rel, uint32_t col, uint64_t s, uint64_t t, char op, uint64_t v, qe_h* out) {
    Eng* e = E(u);
    return guard(e, [&] {
        qe_ctx* c = e->c;
        const qe_col q = column(c, rel, col);
        if (t > q.n || s > t) throw Error(QE_EINVAL, "bad row range");
        const uint64_t n = t - s;
        uint32_t* d = dalloc_t<uint32_t>(c, std::max<uint64_t>(n, 1));
        const uint64_t m = filter_scan2_unordered(c, q.d + s, op, v, q.d + s, op, v, n, (uint32_t)s, d, nullptr);
        *out = H(new_arr(c, d, m, false));
    });
}

int e_scan2(void* u, uint32_t rel, uint32_t col1, char op1, uint64_t v1, uint32_t col2, char op2, uint64_t v2,
            uint64_t s, uint64_t t, int values, qe_h* out) {
    Eng* e = E(u);
    return guard(e, [&] {
        qe_ctx* c = e->c;
        uint64_t kor = 0, kand = 0;
        // the survivors' col1 values come out of the same pass when the plan expects to ask for them
        // (4 more bytes written per survivor)
        const bool vals = (values & 1) && !(getenv("QE_SCAN_VALUES") && getenv("QE_SCAN_VALUES")[0] == '0') &&
                          qe_relation_column_bits(c, (int)rel, (int)col1, &kor, &kand) == 0 && !(kor >> 32);
        const qe_col q1 = column(c, rel, col1), q2 = column(c, rel, col2);
        if (t > q1.n || t > q2.n || s > t) throw Error(QE_EINVAL, "bad row range");
        const uint64_t n = t - s;
        // ... and the survivors' values of the binding's join key column (values >> 8 = 1 + it), read
        // from its u32 copy: the join's key side then widens them with its sort's histogram instead
        // of gathering the column through the list (QE_SCAN_KEYS=0: gathered -- A/B)
        const uint32_t kc = ((uint32_t)values >> 8) & 0xFFu;
        const uint32_t* k32 = nullptr;
        if (kc && !(getenv("QE_SCAN_KEYS") && getenv("QE_SCAN_KEYS")[0] == '0')) {
            const qe_col qk = column(c, rel, kc - 1);
            k32 = narrow_of(c, qk.d, qk.n);
            if (t > qk.n) k32 = nullptr;
        }
        uint32_t* d = dalloc_t<uint32_t>(c, std::max<uint64_t>(n, 1));
        uint32_t* dv = vals ? dalloc_t<uint32_t>(c, std::max<uint64_t>(n, 1)) : nullptr;
        uint32_t* dk = k32 ? dalloc_t<uint32_t>(c, std::max<uint64_t>(n, 1)) : nullptr;
        const uint64_t m = filter_scan2_unordered(c, q1.d + s, op1, v1, q2.d + s, op2, v2, n, (uint32_t)s, d, dv,
                                                  k32 ? k32 + s : nullptr, dk);
        DArr* a = new_arr(c, d, m, false);
        if (vals) {
            a->vcache = dv;
            a->vrel = rel;
            a->vcol = col1;
        }
        if (dk) {
            a->kcache = dk;
            a->krel = rel;
            a->kcol = kc - 1;
        }
        *out = H(a);
    });
}

int e_iota(void* u, uint64_t s, uint64_t n, qe_h* out) {
    Eng* e = E(u);
    return guard(e, [&] {
        qe_list l{};
        ck(qe_iota(e->c, s, n, &l), e->c);
        *out = H(new_arr(e->c, l.d, l.n, false));
    });
}

int e_refine(void* u, uint32_t rel, uint32_t col, qe_h rows, char op, uint64_t v, qe_h* out) {
    Eng* e = E(u);
    return guard(e, [&] {
        DArr* a = A(rows);
        if (a->vcache) {   // the refined list is a different one: its cached values are stale
            dfree(e->c, a->vcache);
            a->vcache = nullptr;
        }
        if (a->kcache) {
            dfree(e->c, a->kcache);
            a->kcache = nullptr;
        }
        qe_list l = as_list(a);
        l.flags = QE_LIST_DISTINCT;
        ck(qe_filter_refine(e->c, column(e->c, rel, col), op, v, &l), e->c);
        a->d = l.d;
        a->n = l.n;
        *out = rows;
    });
}

// the plan engine's key gathers may leave their keys as u32 (PreHist::k32): set for the call only,
// cleared on every exit (a throw included) -- the faithful executor's gathers never see it
struct K32Scope {
    qe_ctx* c;
    explicit K32Scope(qe_ctx* cc) : c(cc) { c->gather_k32 = true; }
    ~K32Scope() { c->gather_k32 = false; }
};

int e_keys(void* u, uint32_t rel, uint32_t col, qe_h rows, qe_h* out) {
    Eng* e = E(u);
    DArr* r = A(rows);
    if (r->kcache && r->krel == rel && r->kcol == col) {   // the scan that made the list emitted the keys
        return guard(e, [&] {
            qe_ctx* c = e->c;
            uint64_t kor = 0, kand = 0;
            ck(qe_relation_column_bits(c, (int)rel, (int)col, &kor, &kand), c);
            const uint64_t n = r->n;
            uint32_t* kv = r->kcache;
            r->kcache = nullptr;
            uint64_t* k = dalloc_t<uint64_t>(c, std::max<uint64_t>(n, 1));
            bool fused = false, adopted = false;
            if (n) {
                K32Scope k32(c);
                fused = widen_with_hist(c, kv, n, kor, kand, k, &adopted);
            }
            if (n && !fused) {
                Timed t(c, "widen_keys", 12.0 * n);
                hipLaunchKernelGGL(widen_u32_kernel, dim3(grid_for(n, 256 * 8, 8192)), dim3(256), 0, c->stream, kv, n, k);
                QE_HIP(hipGetLastError());
            }
            if (!adopted) dfree(c, kv);
            DArr* a = new_arr(c, k, n, true);
            a->bits = true;
            a->kor = kor;
            a->kand = kand;
            *out = H(a);
        });
    }
    return guard(e, [&] {
        qe_list l = as_list(A(rows));
        qe_pairs p{};
        int rc;
        {
            K32Scope k32(e->c);   // the keys go to a join's sort (or an exchange, which widens them)
            rc = qe_gather_pairs(e->c, column(e->c, rel, col), &l, &p);
        }
        ck(rc, e->c);
        DArr* k = new_arr(e->c, p.key, p.n, true);
        k->bits = (p.flags & QE_PAIRS_BITS) != 0;
        k->kor = p.kor;
        k->kand = p.kand;
        *out = H(k);
    });
}

// a base column as a payload: its values ride with the relation's rows through the join
// (join_carry's xa) when all of them fit 32 bits
int e_column(void* u, uint32_t rel, uint32_t col, qe_h* out) {
    Eng* e = E(u);
    qe_ctx* c = e->c;
    uint64_t kor = 0, kand = 0;
    if (qe_relation_column_bits(c, (int)rel, (int)col, &kor, &kand) != 0 || (kor >> 32)) return QE_ENOTSUP;
    return guard(e, [&] {
        const qe_col q = column(c, rel, col);
        DArr* a = new_arr(c, const_cast<uint64_t*>(q.d), q.n, true, false);
        a->colview = true;
        *out = H(a);
    });
}

// keys from the carried values of the key column: widened, with the sort's histogram when the
// sort will take it -- what e_keys computes, without the random gather through the rowids
int e_keys_of(void* u, uint32_t rel, uint32_t col, qe_h vals, qe_h* out) {
    Eng* e = E(u);
    return guard(e, [&] {
        qe_ctx* c = e->c;
        uint64_t kor = 0, kand = 0;
        ck(qe_relation_column_bits(c, (int)rel, (int)col, &kor, &kand), c);
        DArr* v = A(vals);
        const uint64_t n = v->n;
        uint64_t* k = dalloc_t<uint64_t>(c, std::max<uint64_t>(n, 1));
        const uint32_t* vd = static_cast<const uint32_t*>(v->d);
        bool fused;
        {
            K32Scope k32(c);
            // an owned value list (the join's carried key values, released by the plan right after)
            // is handed to the sort as its u32 key copy (no copy written); a borrowed one is copied
            const bool own = v->owned && !v->colview;
            bool adopted = false;
            fused = n && widen_with_hist(c, vd, n, kor, kand, k, own ? &adopted : nullptr);
            if (adopted) v->d = nullptr;   // (the sort's PreHist owns the block now)
        }
        if (n && !fused) {
            Timed t(c, "widen_keys", 12.0 * n);
            hipLaunchKernelGGL(widen_u32_kernel, dim3(grid_for(n, 256 * 8, 8192)), dim3(256), 0, c->stream, vd, n, k);
            QE_HIP(hipGetLastError());
        }
        DArr* a = new_arr(c, k, n, true);
        a->bits = true;
        a->kor = kor;
        a->kand = kand;
        *out = H(a);
    });
}

// the whole column at any rank count (the plan's broadcast joins): as e_base_side at one rank
int e_base_side_all(void* u, uint32_t rel, uint32_t col, qe_h* keys, qe_h* rowids) {
    Eng* e = E(u);
    return guard(e, [&] {
        qe_ctx* c = e->c;
        const qe_col q = column(c, rel, col);
        uint64_t kor = 0, kand = 0;
        ck(qe_relation_column_bits(c, (int)rel, (int)col, &kor, &kand), c);
        DArr* k = new_arr(c, const_cast<uint64_t*>(q.d), q.n, true, false);
        k->bits = true;
        k->kor = kor;
        k->kand = kand;
        *keys = H(k);
        *rowids = 0;
    });
}

int e_base_side(void* u, uint32_t rel, uint32_t col, qe_h* keys, qe_h* rowids) {
    Eng* e = E(u);
    return guard(e, [&] {
        qe_ctx* c = e->c;
        const qe_col q = column(c, rel, col);
        uint64_t kor = 0, kand = 0;
        ck(qe_relation_column_bits(c, (int)rel, (int)col, &kor, &kand), c);
        if (e->world == 1) {                  // the column itself, row i: zero copy
            DArr* k = new_arr(c, const_cast<uint64_t*>(q.d), q.n, true, false);
            k->bits = true;
            k->kor = kor;
            k->kand = kand;
            *keys = H(k);
            *rowids = 0;
            return;
        }
        if (c->bparts_n == (uint32_t)e->world && c->bparts_p == (uint32_t)e->rank) {
            // partitioned layout (qe_partition_columns): this column's bucket is selected the first
            // time a join reads it as a whole base side and kept until the relations are dropped, so
            // only join-key columns ever hold one (columns read only as payloads or by broadcast
            // joins never do)
            auto it = c->bparts.find(q.d);
            if (it == c->bparts.end()) {
                qe_pairs p{};
                bucket_select_dev(c, q, (uint32_t)e->world, (uint32_t)e->rank, nullptr, 0, nullptr, &p);
                it = c->bparts.emplace(q.d, p).first;
                c->load_bytes += 8.0 * (double)q.n + 12.0 * (double)p.n;
            }
            {
                DArr* k = new_arr(c, it->second.key, it->second.n, true, false);
                k->bits = true;
                k->kor = kor;
                k->kand = kand;
                *keys = H(k);
                *rowids = H(new_arr(c, it->second.val, it->second.n, false, false));
                return;
            }
        }
        qe_pairs p{};                          // this rank's hash bucket of the replicated column
        ck(qe_bucket_select(c, q, (uint32_t)e->world, (uint32_t)e->rank, nullptr, 0, &p), c);
        DArr* k = new_arr(c, p.key, p.n, true);
        k->bits = true;
        k->kor = kor;
        k->kand = kand;
        *keys = H(k);
        *rowids = H(new_arr(c, p.val, p.n, false));
    });
}

// partition (ctx stream, no host sync) -> counts all-to-all + the grouped send/recv of every array
// on the comm stream; the ctx stream carries on with the other join side meanwhile.
// Keys below 2^32 (the side's bounds: column statistics, the same on every rank) travel as u32:
// partitioned from the side's pending u32 copy when it has one (PreHist::k32), sent as 4 B a key
// instead of 8, and at the receiver widened only where the join's sort needs it (exchange_finish).
// Every rank's choice rides in the top bit of its count words, checked before any byte moves.
static bool exchange_k32_on() {
    const char* s = getenv("QE_EXCHANGE_K32");   // (A/B: 0 sends u64 keys)
    return !(s && s[0] == '0');
}
constexpr uint64_t K32_FLAG = 1ull << 63;
// marks this rank's send counts (cnt[0, W), after the scatter has read its cursors) as u32 keys
__global__ void __launch_bounds__(64) flag_counts_kernel(unsigned long long* cnt, int W) {
    if ((int)threadIdx.x < W) cnt[threadIdx.x] |= (unsigned long long)K32_FLAG;
}

int e_exchange_start(void* u, qe_h keys, const qe_h* cols, int ncols, qe_h* ticket) {
    Eng* e = E(u);
    return guard(e, [&] {
        qe_ctx* c = e->c;
        qe_comm* m = e->comm;
        const int W = e->world;
        DArr* k = A(keys);
        const uint64_t n = k->n;
        const bool k32 = k->bits && !(k->kor >> 32) && exchange_k32_on();
        const uint32_t* kin32 = k32 ? keys_pending_u32(c, k->d) : nullptr;
        if (!kin32) keys_need_u64(c, k->d);   // (keys gathered as u32 for a sort, sent as u64: widened)
        const size_t kw = k32 ? 4 : 8;
        // more than 4 rowid columns: an index rides through the partition, the columns follow it
        const bool via_idx = ncols > 4;
        std::vector<const uint32_t*> in;
        uint32_t* idx = nullptr;
        if (via_idx) {
            qe_list l{};
            ck(qe_iota(c, 0, n, &l), c);
            idx = l.d;
            in.push_back(idx);
        } else {
            for (int i = 0; i < ncols; i++) in.push_back(static_cast<const uint32_t*>(A(cols[i])->d));
        }
        const int np = (int)in.size();
        void* sk = dalloc(c, std::max<uint64_t>(n, 1) * kw);
        std::vector<uint32_t*> sc(np);
        for (int i = 0; i < np; i++) sc[i] = dalloc_t<uint32_t>(c, std::max<uint64_t>(n, 1));
        unsigned long long* cnt = dalloc_t<unsigned long long>(c, 4 * 64);   // [send | cursors | recv | -]
        partition_dev(c, static_cast<const uint64_t*>(k->d), n, in.data(), np, (uint32_t)W, cnt,
                      static_cast<uint64_t*>(sk), sc.data(), kin32, k32);
        if (k32) {
            hipLaunchKernelGGL(flag_counts_kernel, dim3(1), dim3(64), 0, c->stream, cnt, W);
            QE_HIP(hipGetLastError());
        }
        Ticket* t = new Ticket;
        t->send.push_back(sk);
        for (auto* p : sc) t->send.push_back(p);
        t->send.push_back(cnt);
        std::vector<uint32_t*> scols;                  // the columns in partitioned order
        if (via_idx) {
            for (int i = 0; i < ncols; i++) {
                qe_list il{};
                il.d = sc[0];
                il.n = n;
                qe_list o{};
                ck(qe_take_u32(c, static_cast<const uint32_t*>(A(cols[i])->d), &il, &o), c);
                scols.push_back(o.d);
                t->send.push_back(o.d);
            }
            dfree(c, idx);
        } else {
            scols = sc;
        }
        hipEvent_t ready;
        QE_HIP(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
        QE_HIP(hipEventRecord(ready, c->stream));
        QE_HIP(hipStreamWaitEvent(m->stream, ready, 0));
        QE_HIP(hipEventDestroy(ready));
        uint64_t hc[2 * 64];
        LocalGroup* g = m->local;
        if (g) {   // counts all-to-all: post this rank's send counts and segments, read the peers'
            QE_HIP(hipMemcpyAsync(hc, cnt, 64 * sizeof(uint64_t), hipMemcpyDeviceToHost, m->stream));
            QE_HIP(hipStreamSynchronize(m->stream));   // (the partitioned segments are complete too)
            std::copy(hc, hc + W, g->cnt[e->rank].begin());   // (flagged on the device, as below)
            g->keys[e->rank] = sk;
            g->cols[e->rank].assign(scols.begin(), scols.end());
            g->barrier();
            for (int p = 0; p < W; p++) {
                if ((int)g->cols[p].size() != ncols) throw Error(QE_EINVAL, "internal: ranks exchange different columns");
                hc[64 + p] = g->cnt[p][e->rank];
            }
        } else {
            QE_NCCL(ncclAllToAll(cnt, cnt + 128, 1, ncclUint64, m->comm, m->stream));
            QE_HIP(hipMemcpyAsync(hc, cnt, 64 * sizeof(uint64_t), hipMemcpyDeviceToHost, m->stream));
            QE_HIP(hipMemcpyAsync(hc + 64, cnt + 128, 64 * sizeof(uint64_t), hipMemcpyDeviceToHost, m->stream));
            QE_HIP(hipStreamSynchronize(m->stream));   // the one host round trip: receive sizes
        }
        // every peer must send keys of this rank's width: a mismatch (ranks disagreeing on the
        // switch) is seen by every rank of the exchange -- each has a peer of the other width --
        // so all of them stop here, before the grouped send/recv
        for (int p = 0; p < W; p++) {
            if (((hc[64 + p] & K32_FLAG) != 0) != k32)
                throw Error(QE_EINVAL, "exchange: ranks send keys of different widths (QE_EXCHANGE_K32 differs)");
            hc[p] &= ~K32_FLAG;
            hc[64 + p] &= ~K32_FLAG;
        }
        uint64_t soff[64], roff[64], total = 0, run = 0;
        for (int p = 0; p < W; p++) {
            soff[p] = run;
            run += hc[p];
            roff[p] = total;
            total += hc[64 + p];
        }
        if (run != n) throw Error(QE_EINVAL, "internal: partition counts do not add up");
        void* rkd = dalloc(c, std::max<uint64_t>(total, 1) * kw);
        DArr* rk = new_arr(c, k32 ? nullptr : rkd, total, true);
        if (k32) t->keys32 = rkd;
        rk->bits = k->bits;
        rk->kor = k->kor;
        rk->kand = k->kand;
        t->keys = rk;
        for (int i = 0; i < ncols; i++)
            t->cols.push_back(new_arr(c, dalloc_t<uint32_t>(c, std::max<uint64_t>(total, 1)), total, false));
        if (g) {   // the grouped send/recv: pull segment `rank` of every sender
            for (int p = 0; p < W; p++) {
                const uint64_t nr = hc[64 + p];
                if (!nr) continue;
                uint64_t so = 0;                       // the sender's segment offset for this rank
                for (int q = 0; q < e->rank; q++) so += g->cnt[p][q] & ~K32_FLAG;
                QE_HIP(hipMemcpyAsync(static_cast<char*>(rkd) + roff[p] * kw,
                                      static_cast<const char*>(g->keys[p]) + so * kw, nr * kw,
                                      hipMemcpyDeviceToDevice, m->stream));
                for (int i = 0; i < ncols; i++)
                    QE_HIP(hipMemcpyAsync(static_cast<uint32_t*>(t->cols[i]->d) + roff[p], g->cols[p][i] + so, nr * 4,
                                          hipMemcpyDeviceToDevice, m->stream));
            }
            QE_HIP(hipStreamSynchronize(m->stream));
            g->barrier();                              // every peer has its segments: sends may be freed
        } else {
            const ncclDataType_t kt = k32 ? ncclUint32 : ncclUint64;
            QE_NCCL(ncclGroupStart());
            for (int p = 0; p < W; p++) {
                QE_NCCL(ncclSend(static_cast<char*>(sk) + soff[p] * kw, hc[p], kt, p, m->comm, m->stream));
                QE_NCCL(ncclRecv(static_cast<char*>(rkd) + roff[p] * kw, hc[64 + p], kt, p, m->comm, m->stream));
                for (int i = 0; i < ncols; i++) {
                    QE_NCCL(ncclSend(scols[i] + soff[p], hc[p], ncclUint32, p, m->comm, m->stream));
                    QE_NCCL(ncclRecv(static_cast<uint32_t*>(t->cols[i]->d) + roff[p], hc[64 + p], ncclUint32, p,
                                     m->comm, m->stream));
                }
            }
            QE_NCCL(ncclGroupEnd());
        }
        QE_HIP(hipEventCreateWithFlags(&t->done, hipEventDisableTiming));
        QE_HIP(hipEventRecord(t->done, m->stream));
        m->exchanges++;
        m->bytes_sent += (n - hc[e->rank]) * (kw + 4 * (uint64_t)ncols);
        delete k;                                      // the inputs are consumed
        for (int i = 0; i < ncols; i++) delete A(cols[i]);
        *ticket = H(t);
    });
}

int e_exchange_finish(void* u, qe_h ticket, qe_h* keys, qe_h* cols) {
    Eng* e = E(u);
    return guard(e, [&] {
        qe_ctx* c = e->c;
        Ticket* t = reinterpret_cast<Ticket*>(ticket);
        QE_HIP(hipStreamWaitEvent(c->stream, t->done, 0));   // later ctx work sees the bucket
        QE_HIP(hipEventDestroy(t->done));
        for (void* p : t->send) dfree(c, p);                  // stream-ordered after the wait
        if (t->keys32) {
            // u32 keys received: the join's sort takes them as its u32 copy with their histogram
            // (widen_with_hist adopts the buffer: no copy, the u64 buffer stays unwritten), or
            // they are widened into the u64 buffer
            DArr* rk = t->keys;
            const uint64_t n = rk->n;
            const uint32_t* r32 = static_cast<const uint32_t*>(t->keys32);
            uint64_t* kb = dalloc_t<uint64_t>(c, std::max<uint64_t>(n, 1));
            rk->d = kb;
            bool fused = false, adopted = false;
            if (n) {
                K32Scope k32(c);
                fused = widen_with_hist(c, r32, n, rk->kor, rk->kand, kb, &adopted);
            }
            if (n && !fused) {
                Timed tm(c, "widen_keys", 12.0 * n);
                hipLaunchKernelGGL(widen_u32_kernel, dim3(grid_for(n, 256 * 8, 8192)), dim3(256), 0, c->stream, r32, n,
                                   kb);
                QE_HIP(hipGetLastError());
            }
            if (!adopted) dfree(c, t->keys32);
            t->keys32 = nullptr;
        }
        *keys = H(t->keys);
        for (size_t i = 0; i < t->cols.size(); i++) cols[i] = H(t->cols[i]);
        delete t;
    });
}

qe_pairs side_pairs(const DArr* k, const DArr* v) {
    if (v && v->colview) throw Error(QE_EINVAL, "a column's values as a join side's vals: join_carry only");
    qe_pairs p{};
    p.key = static_cast<uint64_t*>(k->d);
    p.val = v ? static_cast<uint32_t*>(v->d) : nullptr;
    p.n = k->n;
    if (k->bits) {
        p.kor = k->kor;
        p.kand = k->kand;
        p.flags = QE_PAIRS_BITS;
    }
    return p;
}

int e_join(void* u, qe_h ka, qe_h va, qe_h kb, qe_h vb, qe_h* oa, qe_h* ob) {
    Eng* e = E(u);
    return guard(e, [&] {
        qe_ctx* c = e->c;
        qe_pairs P = side_pairs(A(ka), va ? A(va) : nullptr);
        qe_pairs Q = side_pairs(A(kb), vb ? A(vb) : nullptr);
        qe_list la{}, lb{};
        // the plan's pairs need no order (their consumers are joins that sort again, takes and sums)
        static const bool ordered = getenv("QE_PLAN_MERGE") && getenv("QE_PLAN_MERGE")[0] == '1';
        int rc = 0;
        if (ordered) {
            rc = qe_sort_pairs(c, &P);
            if (rc == 0) rc = qe_sort_pairs(c, &Q);
            if (rc == 0) rc = qe_merge_join(c, &P, &Q, &la, &lb);
        } else {
            rc = qe_join_pairs(c, &P, &Q, &la, &lb);
        }
        qe_pairs_free(c, &P);
        qe_pairs_free(c, &Q);
        ck(rc, c);
        *oa = H(new_arr(c, la.d, la.n, false));
        *ob = H(new_arr(c, lb.d, lb.n, false));
    });
}

// the join with b's carried columns: up to two ride through b's sort and the bucket join (S =
// b), and a's payload column (xa: a's next join key) through a's sort (R = a); otherwise (or on a
// bucket beyond LDS) the join runs on b's positions and every column, b's vals included, is taken
// through them, a's payload gathered through a's rowids
int e_join_carry(void* u, qe_h ka, qe_h va, qe_h kb, qe_h vb, int nb, const qe_h* cb, qe_h xa, qe_h* oa, qe_h* ob,
                 qe_h* outb, qe_h* outxa) {
    Eng* e = E(u);
    return guard(e, [&] {
        qe_ctx* c = e->c;
        const DArr* X = xa ? A(xa) : nullptr;
        if (X && !X->colview) throw Error(QE_EINVAL, "join_carry: xa is not a column");
        // va a column (a whole base relation whose binding rides as that column's values): a's
        // rows are its positions, and its sort packs the column's low words in place of them
        const DArr* VC = va && A(va)->colview ? A(va) : nullptr;
        if (VC && A(ka)->n != VC->n) throw Error(QE_EINVAL, "join_carry: vals column of another length");
        qe_pairs P = side_pairs(A(ka), va && !VC ? A(va) : nullptr);
        qe_pairs Q = side_pairs(A(kb), vb ? A(vb) : nullptr);
        qe_list la{}, lb{}, lx0{}, lx1{}, lxa{};
        auto gather_col = [&](const uint32_t* rows, uint64_t n, const DArr* col) {   // a column's values at rowids
            uint32_t* d = dalloc_t<uint32_t>(c, std::max<uint64_t>(n, 1));
            if (n) {
                Timed t(c, "gather_values", 12.0 * n);
                hipLaunchKernelGGL(gather_u32_kernel, dim3(grid_for(n, 256 * 16, 8192)), dim3(256), 0, c->stream,
                                   static_cast<const uint64_t*>(col->d), rows, n, d);
                QE_HIP(hipGetLastError());
            }
            return d;
        };
        if (nb >= 0 && nb <= 2 && (nb >= 1 || X)) {
            // a's payload in a's input order: the column itself (a = the whole column, row i), or
            // its values at a's rowids (a rank's bucket: ascending rows, a near-sequential read)
            const uint64_t* rc64 = X && (!va || VC) ? static_cast<const uint64_t*>(X->d) : nullptr;
            uint32_t* rx32 = X && va && !VC ? gather_col(static_cast<const uint32_t*>(A(va)->d), A(va)->n, X) : nullptr;
            const bool done =
                join_pairs_carry(c, &P, &Q, nb >= 1 ? static_cast<const uint32_t*>(A(cb[0])->d) : nullptr,
                                 nb == 2 ? static_cast<const uint32_t*>(A(cb[1])->d) : nullptr, &la, &lb, &lx0, &lx1,
                                 rx32, rc64, X ? &lxa : nullptr, VC ? static_cast<const uint64_t*>(VC->d) : nullptr);
            dfree(c, rx32);
            if (done) {
                qe_pairs_free(c, &P);
                qe_pairs_free(c, &Q);
                *oa = H(new_arr(c, la.d, la.n, false));
                *ob = H(new_arr(c, lb.d, lb.n, false));
                if (nb >= 1) outb[0] = H(new_arr(c, lx0.d, lx0.n, false));
                if (nb == 2) outb[1] = H(new_arr(c, lx1.d, lx1.n, false));
                if (X) *outxa = H(new_arr(c, lxa.d, lxa.n, false));
                return;
            }
        }
        qe_pairs Qp = side_pairs(A(kb), nullptr);   // b's positions
        const int rc = qe_join_pairs(c, &P, &Qp, &la, &lb);
        qe_pairs_free(c, &P);
        qe_pairs_free(c, &Qp);
        ck(rc, c);
        if (X) *outxa = H(new_arr(c, gather_col(la.d, la.n, X), la.n, false));   // la: a's rowids
        if (VC) {   // a's binding as the column's values
            *oa = H(new_arr(c, gather_col(la.d, la.n, VC), la.n, false));
            dfree(c, la.d);
        } else {
            *oa = H(new_arr(c, la.d, la.n, false));
        }
        auto take = [&](const DArr* src) {
            qe_list o{};
            ck(qe_take_u32(c, static_cast<const uint32_t*>(src->d), &lb, &o), c);
            return H(new_arr(c, o.d, o.n, false));
        };
        for (int k = 0; k < nb; k++) outb[k] = take(A(cb[k]));
        if (vb) {
            *ob = take(A(vb));
            dfree(c, lb.d);
        } else {
            *ob = H(new_arr(c, lb.d, lb.n, false));
        }
    });
}

int e_checksums(void* u, int n, const uint32_t* rels, const uint32_t* cols, const qe_h* rows, uint64_t* sums);
void e_release(void* u, qe_h h);

// the last join, read only by the checksums: its pair count and the sums of the selected columns
// over b's bindings (src 0: b's vals, k: cb[k - 1]) without materialising the pairs
// (bucket_join_sums); otherwise join_carry + the checksums of its lists, released here
int e_join_sums(void* u, qe_h ka, qe_h va, qe_h kb, qe_h vb, int nb, const qe_h* cb, int nsel, const int* src,
                const uint32_t* rels, const uint32_t* cols, uint64_t* pairs, uint64_t* sums) {
    Eng* e = E(u);
    if (nb >= 0 && nb <= 2 && nsel >= 1 && nsel <= HJ_SUMS) {
        bool done = false;
        const int rc = guard(e, [&] {
            qe_ctx* c = e->c;
            HjSums sc{};
            sc.n = nsel;
            for (int s = 0; s < nsel; s++) {   // a value-carrying list is summed, not gathered through
                sc.col[s] = (src[s] & QE_PLAN_VALUES_SRC) ? nullptr : column(c, rels[s], cols[s]).d;
                sc.src[s] = src[s];
            }
            qe_pairs P = side_pairs(A(ka), va ? A(va) : nullptr);
            qe_pairs Q = side_pairs(A(kb), vb ? A(vb) : nullptr);
            // the sort may replace P / Q by buffers of its own: released on every exit, a throw included
            struct Release {
                qe_ctx* c;
                qe_pairs *p, *q;
                ~Release() {
                    qe_pairs_free(c, p);
                    qe_pairs_free(c, q);
                }
            } release{c, &P, &Q};
            done = join_pairs_sums(c, &P, &Q, nb >= 1 ? static_cast<const uint32_t*>(A(cb[0])->d) : nullptr,
                                   nb == 2 ? static_cast<const uint32_t*>(A(cb[1])->d) : nullptr, sc, pairs, sums);
        });
        if (rc != 0 || done) return rc;
    }
    qe_h oa = 0, ob = 0, outb[2] = {0, 0};
    int rc = nb >= 1 ? e_join_carry(u, ka, va, kb, vb, nb, cb, 0, &oa, &ob, outb, nullptr)
                     : e_join(u, ka, va, kb, vb, &oa, &ob);
    if (rc == 0) {
        *pairs = A(oa)->n;
        std::vector<qe_h> rows(nsel);
        std::vector<uint32_t> rl(nsel);
        for (int s = 0; s < nsel; s++) {
            const int k = src[s] & 3;
            rows[s] = k == 0 ? ob : outb[k - 1];
            rl[s] = (src[s] & QE_PLAN_VALUES_SRC) ? QE_PLAN_VALUES : rels[s];
        }
        if (*pairs) rc = e_checksums(u, nsel, rl.data(), cols, rows.data(), sums);
        else
            for (int s = 0; s < nsel; s++) sums[s] = 0;
    }
    for (qe_h h : {oa, ob, outb[0], outb[1]})
        if (h) e_release(u, h);
    return rc;
}

int e_take(void* u, qe_h src, qe_h idx, qe_h* out) {
    Eng* e = E(u);
    return guard(e, [&] {
        qe_list il = as_list(A(idx)), o{};
        ck(qe_take_u32(e->c, static_cast<const uint32_t*>(A(src)->d), &il, &o), e->c);
        *out = H(new_arr(e->c, o.d, o.n, false));
    });
}

int e_length(void* u, qe_h h, uint64_t* n) {
    (void)u;
    *n = A(h)->n;
    return 0;
}

int e_checksums(void* u, int n, const uint32_t* rels, const uint32_t* cols, const qe_h* rows, uint64_t* sums) {
    Eng* e = E(u);
    return guard(e, [&] {
        qe_ctx* c = e->c;
        std::vector<qe_col> cs;
        std::vector<qe_list> ls(n);
        std::vector<const qe_list*> lp;
        std::vector<int> at, vat;
        for (int i = 0; i < n; i++) {
            ls[i] = as_list(A(rows[i]));
            if (rels[i] == QE_PLAN_VALUES) {   // the list holds the select's values: its own sum
                vat.push_back(i);
                continue;
            }
            cs.push_back(column(c, rels[i], cols[i]));
            lp.push_back(&ls[i]);
            at.push_back(i);
        }
        if (!vat.empty()) {
            unsigned long long* d = (unsigned long long*)dalloc_t<uint64_t>(c, vat.size());
            hipLaunchKernelGGL(zero_words_kernel, dim3(1), dim3(64), 0, c->stream, (uint64_t*)d, (int)vat.size());
            QE_HIP(hipGetLastError());
            for (size_t k = 0; k < vat.size(); k++) {
                const qe_list& l = ls[vat[k]];
                if (!l.n) continue;
                Timed t(c, "checksum", 4.0 * l.n);
                hipLaunchKernelGGL(sum_u32_kernel, dim3(grid_for(l.n, 256 * 16, 4096)), dim3(256), 0, c->stream, l.d,
                                   l.n, d + k);
                QE_HIP(hipGetLastError());
            }
            std::vector<uint64_t> h(vat.size());
            read_words(c, (const uint64_t*)d, h.data(), (int)vat.size());
            dfree(c, d);
            for (size_t k = 0; k < vat.size(); k++) sums[vat[k]] = h[k];
        }
        if (!at.empty()) {
            std::vector<uint64_t> h(at.size());
            ck(qe_checksums(c, (int)at.size(), cs.data(), lp.data(), h.data()), c);
            for (size_t k = 0; k < at.size(); k++) sums[at[k]] = h[k];
        }
    });
}

int e_values(void* u, uint32_t rel, uint32_t col, qe_h rows, qe_h* out) {
    Eng* e = E(u);
    qe_ctx* c = e->c;
    uint64_t kor = 0, kand = 0;
    if (qe_relation_column_bits(c, (int)rel, (int)col, &kor, &kand) != 0 || (kor >> 32)) return QE_ENOTSUP;
    return guard(e, [&] {
        DArr* r = A(rows);
        if (r->vcache && r->vrel == rel && r->vcol == col) {   // made by the scan that made the list
            *out = H(new_arr(c, r->vcache, r->n, false));
            r->vcache = nullptr;
            return;
        }
        const qe_col q = column(c, rel, col);
        uint32_t* d = dalloc_t<uint32_t>(c, std::max<uint64_t>(r->n, 1));
        if (r->n) {
            Timed t(c, "gather_values", 12.0 * r->n);
            hipLaunchKernelGGL(gather_u32_kernel, dim3(grid_for(r->n, 256 * 16, 8192)), dim3(256), 0, c->stream, q.d,
                               static_cast<const uint32_t*>(r->d), r->n, d);
            QE_HIP(hipGetLastError());
        }
        *out = H(new_arr(c, d, r->n, false));
    });
}

int e_allreduce(void* u, uint64_t* v, int n) {
    Eng* e = E(u);
    if (!e->comm) return 0;
    for (int i = 0; i < n; i += 64) {                 // (the communicator reduces 64 words at a time)
        const int rc = qe_allreduce_u64(e->c, e->comm, v + i, std::min(64, n - i));
        if (rc) return rc;
    }
    return 0;
}

// the aggregate join's minimum size (both sides' rows), as the faithful executor's (QE_AGG_MIN)
uint64_t agg_min_rows() {
    static const uint64_t v = [] {
        const char* s = getenv("QE_AGG_MIN");
        return s ? strtoull(s, nullptr, 10) : (1ull << 24);
    }();
    return v;
}

#ifndef QE_HEAVY_SAMPLE
#define QE_HEAVY_SAMPLE (1u << 21)
#endif
#ifndef QE_HEAVY_DIV
#define QE_HEAVY_DIV 64
#endif
#ifndef QE_HEAVY_MAX
#define QE_HEAVY_MAX 32
#endif

// the last join of two whole base relations in aggregate form (C5; SURVEY.md §8(e) "Skew").  One
// rank: qe_join_aggregate's sorts + counting pass.  N ranks, every rank holding both columns:
//   heavy keys -- those whose run in the first QE_HEAVY_SAMPLE rows of either key column is longer
//                 than sample / (N * QE_HEAVY_DIV) (the same list on every rank): each rank counts
//                 them over its row slice of both sides, the counts are all-reduced, and the rank
//                 adds sum_{r in its slice, key heavy} val(r) * |other side's key run|; rank 0 adds
//                 sum_h cA_h * cB_h pairs -- no heavy row moves, no rank takes a whole Zipf head;
//   light keys -- each rank's hash bucket of both columns without the heavy keys
//                 (qe_bucket_select, the select column's low words beside each key), joined in
//                 aggregate form locally.
// The plan all-reduces the shares.
int e_join_agg(void* u, uint32_t ra, uint32_t ca, uint32_t rb, uint32_t cb, int nsel, const int* side,
               const uint32_t* cols, uint64_t* pairs, uint64_t* sums) {
    Eng* e = E(u);
    qe_ctx* c = e->c;
    int vc[2] = {-1, -1};                             // each side's one select column
    for (int s = 0; s < nsel; s++) {
        const int sd = side[s] ? 1 : 0;
        if (vc[sd] >= 0 && vc[sd] != (int)cols[s]) return QE_ENOTSUP;
        vc[sd] = (int)cols[s];
    }
    const uint32_t rel[2] = {ra, rb}, kcol[2] = {ca, cb};
    uint64_t kb[2][2], rows[2];
    for (int sd = 0; sd < 2; sd++) {
        if (qe_relation_rows(c, (int)rel[sd], &rows[sd]) != 0) return QE_ENOTSUP;
        if (rows[sd] >= 0xFFFFFFFFull) return QE_ENOTSUP;
        if (qe_relation_column_bits(c, (int)rel[sd], (int)kcol[sd], &kb[sd][0], &kb[sd][1]) != 0) return QE_ENOTSUP;
        uint64_t vor = 0, vand = 0;
        if (vc[sd] >= 0 && (qe_relation_column_bits(c, (int)rel[sd], vc[sd], &vor, &vand) != 0 || (vor >> 32)))
            return QE_ENOTSUP;
    }
    const uint64_t vary = (kb[0][0] | kb[1][0]) & ~(kb[0][1] & kb[1][1]);
    if (vary && 64 - __builtin_clzll(vary) - __builtin_ctzll(vary) > 32) return QE_ENOTSUP;
    if (rows[0] + rows[1] < agg_min_rows()) return QE_ENOTSUP;
    return guard(e, [&] {
        const qe_col key[2] = {column(c, ra, ca), column(c, rb, cb)};
        qe_col val[2] = {{nullptr, 0}, {nullptr, 0}};
        for (int sd = 0; sd < 2; sd++)
            if (vc[sd] >= 0) val[sd] = column(c, rel[sd], (uint32_t)vc[sd]);
        uint64_t out[3] = {0, 0, 0}, wsum[2] = {0, 0}, heavy_pairs = 0;
        if (e->world == 1) {
            AggSide A{key[0].d, val[0].d, nullptr, key[0].n, {kb[0][0], kb[0][1]}};
            AggSide B{key[1].d, val[1].d, nullptr, key[1].n, {kb[1][0], kb[1][1]}};
            join_aggregate_sides(c, A, B, out);
        } else {
            const std::vector<uint64_t> heavy =
                heavy_keys_dev(c, key, 2, QE_HEAVY_SAMPLE, (uint64_t)e->world * QE_HEAVY_DIV, QE_HEAVY_MAX);
            const uint32_t nh = (uint32_t)heavy.size();
            qe_pairs lp[2] = {};
            struct Release {
                qe_ctx* c;
                qe_pairs* p;
                ~Release() {
                    qe_pairs_free(c, &p[0]);
                    qe_pairs_free(c, &p[1]);
                }
            } release{c, lp};
            for (int sd = 0; sd < 2; sd++)
                bucket_select_dev(c, key[sd], (uint32_t)e->world, (uint32_t)e->rank, heavy.data(), nh, val[sd].d,
                                  &lp[sd]);
            AggSide A{lp[0].key, nullptr, val[0].d ? lp[0].val : nullptr, lp[0].n, {kb[0][0], kb[0][1]}};
            AggSide B{lp[1].key, nullptr, val[1].d ? lp[1].val : nullptr, lp[1].n, {kb[1][0], kb[1][1]}};
            join_aggregate_sides(c, A, B, out);
            if (nh) {
                uint64_t s0[2], s1[2];
                std::vector<uint64_t> cnt(2 * (size_t)nh);   // [this rank's slice counts of A | of B]
                for (int sd = 0; sd < 2; sd++) {
                    s0[sd] = rows[sd] * (uint64_t)e->rank / (uint64_t)e->world;
                    s1[sd] = rows[sd] * (uint64_t)(e->rank + 1) / (uint64_t)e->world;
                    ck(qe_heavy_stats(c, key[sd], s0[sd], s1[sd], heavy.data(), nh, qe_col{nullptr, 0}, nullptr,
                                      cnt.data() + sd * nh, nullptr),
                       c);
                }
                ck(e_allreduce(u, cnt.data(), 2 * (int)nh), c);   // the heavy keys' global counts
                for (uint32_t h = 0; h < nh; h++) heavy_pairs += cnt[h] * cnt[nh + h];
                for (int sd = 0; sd < 2; sd++)
                    if (val[sd].d)
                        ck(qe_heavy_stats(c, key[sd], s0[sd], s1[sd], heavy.data(), nh, val[sd],
                                          cnt.data() + (1 - sd) * nh, nullptr, &wsum[sd]),
                           c);
            }
        }
        *pairs = out[0] + (e->rank == 0 ? heavy_pairs : 0);
        const uint64_t sum[2] = {out[1] + wsum[0], out[2] + wsum[1]};
        for (int s = 0; s < nsel; s++) sums[s] = sum[side[s] ? 1 : 0];
    });
}

void e_release(void* u, qe_h h) {
    (void)u;
    if (h) delete reinterpret_cast<Obj*>(h);
}

// a query outside the plan's domain: the faithful executor on rank 0 (relations are replicated);
// its status reaches every rank so all stop together where the reference exits
int e_fallback(void* u, void* query, void* out) {
    Eng* e = E(u);
    e->refused++;
    int rc = 0;
    if (e->rank == 0) rc = qe_exec_query(e->c, static_cast<query_t*>(query), static_cast<FILE*>(out));
    if (e->comm) {
        uint64_t v = (uint64_t)(int64_t)rc;
        int r2 = e_allreduce(u, &v, 1);
        if (r2) return r2;
        rc = (int)(int64_t)v;
    }
    return rc;
}

// RCCL prints a version banner on stdout when a communicator is made; stdout is the reference's
// protocol channel (main/queries_main.c), so library chatter is sent to stderr meanwhile
struct StdoutToStderr {
    int saved = -1;
    StdoutToStderr() {
        fflush(stdout);
        saved = dup(1);
        if (saved >= 0) dup2(2, 1);
    }
    ~StdoutToStderr() {
        fflush(stdout);
        if (saved >= 0) {
            dup2(saved, 1);
            close(saved);
        }
    }
};

// libqe's engine for the partitioned plan (include/qe_plan.h)
qe_engine make_engine(Eng* e) {
    qe_engine g{};
    g.u = e;
    g.rank = (uint32_t)e->rank;
    g.world = (uint32_t)e->world;
    g.rel_count = e_rel_count;
    g.rel_shape = e_rel_shape;
    g.scan = e_scan;
    g.iota = e_iota;
    g.refine = e_refine;
    g.scan2 = e_scan2;
    g.keys = e_keys;
    g.base_side = e_base_side;
    g.base_side_all = e_base_side_all;
    g.exchange_start = e_exchange_start;
    g.exchange_finish = e_exchange_finish;
    g.join = e_join;
    g.take = e_take;
    g.join_carry = e_join_carry;
    // the last join in aggregate form (QE_PLAN_AGG=0: materialised, then summed -- A/B)
    g.join_sums = getenv("QE_PLAN_AGG") && getenv("QE_PLAN_AGG")[0] == '0' ? nullptr : e_join_sums;
    // select values carried instead of rowids (QE_PLAN_VALUES=0: rowids -- A/B)
    g.values = getenv("QE_PLAN_VALUES") && getenv("QE_PLAN_VALUES")[0] == '0' ? nullptr : e_values;
    g.length = e_length;
    g.checksums = e_checksums;
    g.allreduce = e_allreduce;
    g.release = e_release;
    g.fallback = e_fallback;
    g.mat_limit = &e->c->mat_limit;
    // the last join of two base relations in aggregate form (QE_PLAN_JOIN_AGG=0: as other joins -- A/B)
    g.join_agg = getenv("QE_PLAN_JOIN_AGG") && getenv("QE_PLAN_JOIN_AGG")[0] == '0' ? nullptr : e_join_agg;
    // a base relation's next join key rides with its rows (QE_PLAN_KEY_CARRY=0: gathered -- A/B)
    if (!(getenv("QE_PLAN_KEY_CARRY") && getenv("QE_PLAN_KEY_CARRY")[0] == '0')) {
        g.column = e_column;
        g.keys_of = e_keys_of;
    }
    return g;
}

}  // namespace
}  // namespace qe

using namespace qe;

extern "C" {

int qe_comm_unique_id(uint8_t* id) {
    StdoutToStderr quiet;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return QE_EHIP;
    std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    return 0;
}

int qe_comm_init(qe_ctx* c, int nranks, int rank, const uint8_t* id, qe_comm** out) {
    QE_API_BEGIN(c)
    if (nranks < 1 || nranks > 64 || rank < 0 || rank >= nranks) throw Error(QE_EINVAL, "bad rank / world");
    QE_HIP(hipSetDevice(c->device));
    qe_comm* m = new qe_comm;
    m->nranks = nranks;
    m->rank = rank;
    try {
        ncclUniqueId u;
        std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
        {
            StdoutToStderr quiet;
            QE_NCCL(ncclCommInitRank(&m->comm, nranks, u, rank));
        }
        QE_HIP(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking));
        QE_HIP(hipMalloc(&m->d_red, 64 * sizeof(uint64_t)));
        QE_HIP(hipHostMalloc(&m->h_red, 64 * sizeof(uint64_t), hipHostMallocDefault));
    } catch (...) {
        qe_comm_fini(m);
        throw;
    }
    *out = m;
    return 0;
    QE_API_END(c)
}

int qe_comm_init_local(qe_ctx* const* ctxs, int nranks, qe_comm** out) {
    qe_ctx* c0 = ctxs && nranks > 0 ? ctxs[0] : nullptr;
    QE_API_BEGIN(c0)
    if (!c0 || nranks < 1 || nranks > 64) throw Error(QE_EINVAL, "1..64 ranks, one ctx each");
    for (int r = 0; r < nranks; r++) {
        if (!ctxs[r]) throw Error(QE_EINVAL, "null ctx");
        out[r] = nullptr;
    }
    LocalGroup* g = new LocalGroup;
    g->n = nranks;
    g->red.resize(nranks);
    g->cnt.resize(nranks);
    g->keys.assign(nranks, nullptr);
    g->cols.resize(nranks);
    if (const char* t = getenv("QE_LOCAL_TIMEOUT_S")) g->timeout_s = atof(t);
    try {
        for (int r = 0; r < nranks; r++) {
            qe_comm* m = new qe_comm;
            m->nranks = nranks;
            m->rank = r;
            m->local = g;
            g->refs++;
            out[r] = m;
            QE_HIP(hipSetDevice(ctxs[r]->device));
            QE_HIP(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking));
        }
    } catch (...) {
        if (g->refs == 0) delete g;            // else the last qe_comm_fini deletes it
        for (int r = 0; r < nranks; r++)
            if (out[r]) qe_comm_fini(out[r]);
        throw;
    }
    return 0;
    QE_API_END(c0)
}

int qe_run_queries_local(qe_ctx* c, int nranks, const char* text, char** out, size_t* outlen, uint64_t* refused,
                         uint64_t* bytes_sent) {
    QE_API_BEGIN(c)
    *out = nullptr;
    *outlen = 0;
    if (nranks < 1 || nranks > 16) throw Error(QE_EINVAL, "1..16 in-process ranks");
    qe_ctx* w[16];
    ck(qe_workers(c, nranks, w), c);
    // each rank's buckets of the base columns, as the RCCL ranks take them at load (kept in the
    // worker contexts until the relations are dropped)
    for (int r = 0; r < nranks; r++)
        if (nranks > 1 && (w[r]->bparts_n != (uint32_t)nranks || w[r]->bparts_p != (uint32_t)r))
            ck(qe_partition_columns(w[r], (uint32_t)nranks, (uint32_t)r), w[r]);
    qe_comm* m[16];
    ck(qe_comm_init_local(w, nranks, m), w[0]);
    std::vector<char*> outs(nranks, nullptr);
    std::vector<size_t> lens(nranks, 0);
    std::vector<uint64_t> ref(nranks, 0);
    std::vector<int> rcs(nranks, 0);
    std::vector<std::thread> th;
    for (int r = 0; r < nranks; r++)
        th.emplace_back([&, r] {
            qe_bind_thread(w[r]);
            rcs[r] = qe_run_queries_dist(w[r], m[r], text, &outs[r], &lens[r], &ref[r]);
            if (rcs[r] != 0 && rcs[r] != QE_EEXIT) m[r]->local->fail();   // never leave a peer waiting
        });
    for (auto& t : th) t.join();
    uint64_t sent = 0;
    for (int r = 0; r < nranks; r++) {
        uint64_t x = 0, b = 0;
        qe_comm_stats(m[r], &x, &b);
        sent += b;
        qe_comm_fini(m[r]);
    }
    if (bytes_sent) *bytes_sent = sent;
    if (refused) *refused = ref[0];
    c->last_result_rows = w[0]->last_result_rows;
    int rc = rcs[0];
    for (int r = 0; r < nranks && rc == 0; r++)
        if (rcs[r] != 0) rc = rcs[r];
    for (int r = 0; r < nranks; r++)
        if (rcs[r] != 0 && rcs[r] != QE_EEXIT) {
            c->err = "rank " + std::to_string(r) + ": " + w[r]->err;
            rc = rcs[r];
            break;
        }
    for (int r = 1; r < nranks; r++) free(outs[r]);
    *out = outs[0];
    *outlen = lens[0];
    return rc;
    QE_API_END(c)
}

void qe_comm_fini(qe_comm* m) {
    if (!m) return;
    if (m->stream) (void)hipStreamSynchronize(m->stream);
    if (m->local) {
        LocalGroup* g = m->local;
        bool last;
        {
            std::lock_guard<std::mutex> lk(g->mu);
            last = --g->refs == 0;
        }
        if (last) delete g;
    }
    if (m->comm) {
        StdoutToStderr quiet;
        ncclCommDestroy(m->comm);
    }
    if (m->stream) (void)hipStreamDestroy(m->stream);
    if (m->d_red) (void)hipFree(m->d_red);
    if (m->h_red) (void)hipHostFree(m->h_red);
    delete m;
}

int qe_allreduce_u64(qe_ctx* c, qe_comm* m, uint64_t* vals, int n) {
    QE_API_BEGIN(c)
    if (n < 0 || n > 64) throw Error(QE_EINVAL, "at most 64 values per all-reduce");
    if (!m || n == 0) return 0;        // (one rank still goes through RCCL: the tested path)
    if (LocalGroup* g = m->local) {    // in-process ranks: post, sum every rank's values, release
        try {
            std::copy(vals, vals + n, g->red[m->rank].begin());
            g->barrier();
            for (int i = 0; i < n; i++) {
                uint64_t s = 0;
                for (int p = 0; p < g->n; p++) s += g->red[p][i];
                vals[i] = s;
            }
            g->barrier();
        } catch (...) {
            g->fail();
            throw;
        }
        return 0;
    }
    std::memcpy(m->h_red, vals, n * sizeof(uint64_t));
    // every RCCL call of the communicator goes on its one stream (so no two of them can run in a
    // different order on two ranks); the values are host numbers, nothing to wait for on the ctx
    QE_HIP(hipMemcpyAsync(m->d_red, m->h_red, n * sizeof(uint64_t), hipMemcpyHostToDevice, m->stream));
    QE_NCCL(ncclAllReduce(m->d_red, m->d_red, n, ncclUint64, ncclSum, m->comm, m->stream));
    QE_HIP(hipMemcpyAsync(m->h_red, m->d_red, n * sizeof(uint64_t), hipMemcpyDeviceToHost, m->stream));
    QE_HIP(hipStreamSynchronize(m->stream));
    std::memcpy(vals, m->h_red, n * sizeof(uint64_t));
    return 0;
    QE_API_END(c)
}

int qe_shuffle_pairs(qe_ctx* c, qe_comm* m, const uint64_t* keys, uint64_t n, const uint32_t* const* cols, int ncols,
                     uint64_t** out_keys, uint32_t** out_cols, uint64_t* out_n) {
    QE_API_BEGIN(c)
    if (!m) throw Error(QE_EINVAL, "no communicator");
    if (ncols < 0 || ncols > 64) throw Error(QE_EINVAL, "at most 64 rowid columns");
    Eng e{c, m, m->nranks, m->rank, 0};
    // the engine consumes its inputs: hand it copies it may free, the caller keeps its arrays
    DArr* k = new_arr(c, dalloc_t<uint64_t>(c, std::max<uint64_t>(n, 1)), n, true);
    if (n) QE_HIP(hipMemcpyAsync(k->d, keys, n * 8, hipMemcpyDeviceToDevice, c->stream));
    std::vector<qe_h> hc(ncols);
    for (int i = 0; i < ncols; i++) {
        DArr* a = new_arr(c, dalloc_t<uint32_t>(c, std::max<uint64_t>(n, 1)), n, false);
        if (n) QE_HIP(hipMemcpyAsync(a->d, cols[i], n * 4, hipMemcpyDeviceToDevice, c->stream));
        hc[i] = H(a);
    }
    qe_h t = 0, rk = 0;
    std::vector<qe_h> rc(ncols);
    ck(e_exchange_start(&e, H(k), hc.data(), ncols, &t), c);
    ck(e_exchange_finish(&e, t, &rk, rc.data()), c);
    DArr* K = A(rk);
    *out_keys = static_cast<uint64_t*>(K->d);
    *out_n = K->n;
    K->owned = false;
    delete K;
    for (int i = 0; i < ncols; i++) {
        DArr* a = A(rc[i]);
        out_cols[i] = static_cast<uint32_t*>(a->d);
        a->owned = false;
        delete a;
    }
    QE_HIP(hipStreamSynchronize(c->stream));
    return 0;
    QE_API_END(c)
}

void qe_buffer_free(qe_ctx* c, void* p) {
    if (c && p) dfree(c, p);
}

int qe_comm_stats(qe_comm* m, uint64_t* exchanges, uint64_t* bytes_sent) {
    if (!m) return QE_EINVAL;
    if (exchanges) *exchanges = m->exchanges;
    if (bytes_sent) *bytes_sent = m->bytes_sent;
    return 0;
}

int qe_run_queries_dist(qe_ctx* c, qe_comm* m, const char* text, char** out, size_t* outlen, uint64_t* refused) {
    if (!c) return QE_EINVAL;
    Eng e{c, m, m ? m->nranks : 1, m ? m->rank : 0, 0};
    qe_engine g = make_engine(&e);
    uint64_t rows = c->last_result_rows, nref = 0;
    int rc = qe_plan_run_text(&g, text, out, outlen, &rows, &nref);
    if (refused) *refused = nref;
    c->last_result_rows = rows;
    return rc;
}

int qe_plan_exec_query(qe_ctx* c, query_t* q, FILE* out) {
    Eng e{c, nullptr, 1, 0, 0};
    qe_engine g = make_engine(&e);
    uint64_t rows = c->last_result_rows;
    int refused = 0;
    const int rc = qe_plan_run_query(&g, q, out, &rows, &refused);
    c->last_result_rows = rows;
    return rc;
}

}  // extern "C"
