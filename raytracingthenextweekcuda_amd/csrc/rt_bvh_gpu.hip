// rt_bvh_gpu.hip — the reference's binned-SAH BVH builder on the GPU.
//
// Restates CreateBVH + Recurse + CreateCFBVH / PopulateCacheFriendlyBVH
// (BVH.cpp:94-497, host restatement in rt_bvh.cpp) level by level, one
// workgroup per node of the current level, and produces the same
// CacheFriendlyBVHNode array and triangle list byte for byte:
//
//  * a node's entries are a contiguous segment; the split is a STABLE
//    partition (left, then right, each in work order), so after the last level
//    the entry array lists the leaves in depth-first, left-first order — the
//    order PopulateCacheFriendlyBVH appends them to the triangle list;
//  * the split candidates of an axis are generated with the reference's own
//    float recurrence (split = start + step; split < stop - step; split += step)
//    by one lane, so they are the same floats;
//  * an entry with centre c is left of candidate k iff c < split_k; with the
//    candidates ascending this is k >= bin(c) = #{k : split_k <= c}, so the
//    left set of every candidate is a prefix of a histogram over bins: counts
//    and boxes per bin, then prefix / suffix unions give nl, nr and both boxes;
//  * box unions are min / max, exact and order-free once no coordinate is -0.0
//    (the reference's min3/max3 keep the LAST of equal values, which only shows
//    for -0.0 vs +0.0; the host driver declines such inputs and the caller uses
//    the host builder); LDS atomics run on an order-preserving u32 image of the
//    floats;
//  * the SAH costs use the reference's float expressions (-ffp-contract=off),
//    and the arg-min keeps the first (axis, candidate) with the minimal cost
//    strictly below the node's own cost — the reference's sequential strict `<`.
//
// Depth-first numbering is a second phase: subtree sizes bottom-up per level,
// then DFS indices top-down (root 0, left = parent + 1, right = parent + 1 +
// size(left)), then one pass writes the 32 B nodes.
#include <hip/hip_runtime.h>

#include <float.h>
#include <math.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>

#include "rt_bvh.h"

namespace rt {

namespace {

constexpr int kMaxCand = 1024;  // candidates per axis: 1024 / (depth + 1) - 2 at most

struct Ent {  // BBoxTmp (BVH.cpp:61-76)
    float c[3];
    float lo[3];
    float hi[3];
    int32_t tri;
};

struct PNode {  // one node of the build pool
    int32_t begin, count, level;
    int32_t left, right;  // pool ids, -1 for a leaf
    float lo[3], hi[3];
};

// order-preserving u32 image of a float (no NaN, no -0.0 in the inputs)
__device__ __forceinline__ uint32_t f2o(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float o2f(uint32_t o) {
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o);
}

// min3 / max3 over a triangle's three vertices from FLT_MAX seeds (rt_bvh.cpp build_cf_bvh).
__global__ __launch_bounds__(256) void tri_entries(const float* __restrict__ v, const uint32_t* __restrict__ idx,
                                                   int32_t n, Ent* __restrict__ out) {
    const int32_t j = blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int k = 0; k < 3; ++k) {
        const float* p = v + 3 * (size_t)idx[3 * (size_t)j + k];
        for (int a = 0; a < 3; ++a) {
            lo[a] = lo[a] < p[a] ? lo[a] : p[a];
            hi[a] = hi[a] > p[a] ? hi[a] : p[a];
        }
    }
    Ent e;
    for (int a = 0; a < 3; ++a) {
        e.lo[a] = lo[a];
        e.hi[a] = hi[a];
        e.c[a] = (hi[a] + lo[a]) * 0.5f;  // scale(add(top, bottom), 0.5f)
    }
    e.tri = j;
    out[j] = e;
}

__global__ __launch_bounds__(256) void box_entries(const float* __restrict__ lo, const float* __restrict__ hi,
                                                   int32_t n, Ent* __restrict__ out) {
    const int32_t j = blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    Ent e;
    for (int a = 0; a < 3; ++a) {
        e.lo[a] = lo[3 * (size_t)j + a];
        e.hi[a] = hi[3 * (size_t)j + a];
        e.c[a] = (e.hi[a] + e.lo[a]) * 0.5f;
    }
    e.tri = j;
    out[j] = e;
}

// (count, box) of a run of bins; combine = add / min / max (order-free).
struct Agg {
    uint32_t cnt;
    uint32_t lo[3], hi[3];
};
__device__ __forceinline__ Agg agg_empty() {
    Agg a;
    a.cnt = 0;
    for (int k = 0; k < 3; ++k) {
        a.lo[k] = f2o(FLT_MAX);
        a.hi[k] = f2o(-FLT_MAX);
    }
    return a;
}
__device__ __forceinline__ Agg agg_join(const Agg& a, const Agg& b) {
    Agg r;
    r.cnt = a.cnt + b.cnt;
    for (int k = 0; k < 3; ++k) {
        r.lo[k] = min(a.lo[k], b.lo[k]);
        r.hi[k] = max(a.hi[k], b.hi[k]);
    }
    return r;
}

template <int T, int MC>
struct SplitLds {
    float cand[3][MC];
    int32_t ncand[3];
    float start[3], step[3];
    uint32_t cnt[MC + 1];
    uint32_t blo[3][MC + 1], bhi[3][MC + 1];  // per-bin box, then prefix unions
    uint32_t slo[3][MC + 2], shi[3][MC + 2];  // suffix unions (slot ncand+1 = empty)
    Agg scan[T];
    float red_cost[T];
    uint32_t red_key[T];
    uint32_t wave_tot[T / 64];
    uint32_t box[6];
    float best_cost;
    uint32_t best_key;
    float best_split;
    uint32_t best_nl;
};

__device__ __forceinline__ bool better(float c, uint32_t k, float bc, uint32_t bk) {
    return c < bc || (c == bc && k < bk);
}

// Block-wide inclusive scan of one Agg per thread (Hillis-Steele in LDS).
template <int T, int MC>
__device__ __forceinline__ Agg block_scan(SplitLds<T, MC>& S, Agg v, int tid) {
    S.scan[tid] = v;
    __syncthreads();
    for (int off = 1; off < T; off <<= 1) {
        Agg o = v;
        if (tid >= off) o = agg_join(S.scan[tid - off], v);
        __syncthreads();
        S.scan[tid] = o;
        v = o;
        __syncthreads();
    }
    return v;
}

// One workgroup of T threads per node of the level: box, split search, stable
// partition, children. MC bounds the candidates per axis (1024 / (depth + 1) - 2,
// so 128 from depth 8 on); flags[0] |= 1 if a node needed more.
template <int T, int MC>
__global__ __launch_bounds__(T) void split_level(PNode* __restrict__ pool, int32_t level_begin,
                                                 const Ent* __restrict__ in, Ent* __restrict__ out,
                                                 int32_t* __restrict__ tri_list, int32_t* __restrict__ pool_count,
                                                 int32_t leaf_min_split, int32_t* __restrict__ flags) {
    __shared__ SplitLds<T, MC> S;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    PNode& nd = pool[level_begin + blockIdx.x];
    const int32_t b = nd.begin, n = nd.count, depth = nd.level;
    // blocked assignment: thread t owns entries [t * per, (t + 1) * per), so the
    // 64 lanes of an LDS atomic hit 64 distant (rarely equal) bins
    const int32_t per = (n + T - 1) / T;
    const int32_t i_begin = min(n, tid * per), i_end = min(n, i_begin + per);

    // node box (the parent's lb/lt, or CreateBVH's overall box for the root)
    if (tid < 3) {
        S.box[tid] = f2o(FLT_MAX);
        S.box[3 + tid] = f2o(-FLT_MAX);
    }
    __syncthreads();
    {
        uint32_t l0 = f2o(FLT_MAX), l1 = l0, l2 = l0, h0 = f2o(-FLT_MAX), h1 = h0, h2 = h0;
        for (int32_t i = tid; i < n; i += T) {
            const Ent& e = in[b + i];
            l0 = min(l0, f2o(e.lo[0]));
            l1 = min(l1, f2o(e.lo[1]));
            l2 = min(l2, f2o(e.lo[2]));
            h0 = max(h0, f2o(e.hi[0]));
            h1 = max(h1, f2o(e.hi[1]));
            h2 = max(h2, f2o(e.hi[2]));
        }
        atomicMin(&S.box[0], l0);
        atomicMin(&S.box[1], l1);
        atomicMin(&S.box[2], l2);
        atomicMax(&S.box[3], h0);
        atomicMax(&S.box[4], h1);
        atomicMax(&S.box[5], h2);
    }
    __syncthreads();
    const float bot[3] = {o2f(S.box[0]), o2f(S.box[1]), o2f(S.box[2])};
    const float top[3] = {o2f(S.box[3]), o2f(S.box[4]), o2f(S.box[5])};
    if (tid == 0) {
        for (int a = 0; a < 3; ++a) {
            nd.lo[a] = bot[a];
            nd.hi[a] = top[a];
        }
    }
    auto make_leaf = [&]() {
        for (int32_t i = tid; i < n; i += T) tri_list[b + i] = in[b + i].tri;
        if (tid == 0) {
            nd.left = -1;
            nd.right = -1;
        }
    };
    if (n < leaf_min_split) {  // Recurse: work.size() < 4 -> leaf (BVH.cpp:106)
        make_leaf();
        return;
    }
    // the three axes' candidate sequences, one lane of a different wave each
    const int gen_axis = T >= 192 ? ((tid & 63) == 0 && wave < 3 ? wave : -1) : (tid < 3 ? tid : -1);
    if (gen_axis >= 0) {
        const int axis = gen_axis;
        const float start = bot[axis], stop = top[axis];
        int32_t k = 0;
        if (!((double)fabsf(stop - start) < 1e-4)) {  // BVH.cpp:164
            const float step = (stop - start) / (1024.0f / ((float)depth + 1.0f));
            S.start[axis] = start;
            S.step[axis] = step;
            for (float split = start + step; split < stop - step; split += step) {
                if (k == MC) {
                    atomicOr(flags, 1);
                    break;
                }
                S.cand[axis][k++] = split;
            }
        }
        S.ncand[axis] = k;
    }
    if (tid == 0) {
        const float side1 = top[0] - bot[0], side2 = top[1] - bot[1], side3 = top[2] - bot[2];
        S.best_cost = (float)n * (side1 * side2 + side2 * side3 + side3 * side1);
        S.best_key = 0xFFFFFFFFu;
    }

    for (int axis = 0; axis < 3; ++axis) {
        __syncthreads();
        const int32_t nc = S.ncand[axis];
        if (nc == 0) continue;
        const float* cand = S.cand[axis];
        for (int32_t i = tid; i <= nc; i += T) {
            S.cnt[i] = 0;
            for (int a = 0; a < 3; ++a) {
                S.blo[a][i] = f2o(FLT_MAX);
                S.bhi[a][i] = f2o(-FLT_MAX);
            }
        }
        __syncthreads();
        // histogram: bin(c) = #{k : cand[k] <= c}
        for (int32_t i = i_begin; i < i_end; ++i) {
            const Ent& e = in[b + i];
            const float c = e.c[axis];
            // first k with cand[k] > c: candidate k is about start + (k + 1) * step, so
            // start from that estimate and walk to the exact position (non-decreasing cand)
            const float q = (c - S.start[axis]) / S.step[axis];
            int32_t lo = q > 0.0f ? (q < (float)nc ? (int32_t)q : nc) : 0;
            while (lo < nc && cand[lo] <= c) ++lo;
            while (lo > 0 && cand[lo - 1] > c) --lo;
            atomicAdd(&S.cnt[lo], 1u);
            for (int a = 0; a < 3; ++a) {
                atomicMin(&S.blo[a][lo], f2o(e.lo[a]));
                atomicMax(&S.bhi[a][lo], f2o(e.hi[a]));
            }
        }
        __syncthreads();
        // prefix unions (in place) and suffix unions over bins 0..nc, thread t owning
        // the run [t * bp, (t + 1) * bp)
        const int32_t nb = nc + 1, bp = (nb + T - 1) / T;
        const int32_t j0 = min(nb, tid * bp), j1 = min(nb, j0 + bp);
        Agg run = agg_empty();
        for (int32_t j = j0; j < j1; ++j) {
            Agg x;
            x.cnt = S.cnt[j];
            for (int a = 0; a < 3; ++a) {
                x.lo[a] = S.blo[a][j];
                x.hi[a] = S.bhi[a][j];
            }
            run = agg_join(run, x);
        }
        block_scan<T, MC>(S, run, tid);
        Agg pre = tid > 0 ? S.scan[tid - 1] : agg_empty();  // runs 0..t-1
        __syncthreads();
        block_scan<T, MC>(S, run, T - 1 - tid);  // reversed: thread t sits at slot T-1-t
        Agg suf = tid < T - 1 ? S.scan[T - 2 - tid] : agg_empty();  // runs t+1..T-1
        __syncthreads();
        // suffix within the run (backwards), then prefix within the run (forwards, in place)
        for (int32_t j = j1 - 1; j >= j0; --j) {
            for (int a = 0; a < 3; ++a) {
                suf.lo[a] = min(suf.lo[a], S.blo[a][j]);
                suf.hi[a] = max(suf.hi[a], S.bhi[a][j]);
                S.slo[a][j] = suf.lo[a];
                S.shi[a][j] = suf.hi[a];
            }
        }
        if (tid == 0)
            for (int a = 0; a < 3; ++a) {
                S.slo[a][nb] = f2o(FLT_MAX);
                S.shi[a][nb] = f2o(-FLT_MAX);
            }
        for (int32_t j = j0; j < j1; ++j) {
            pre.cnt += S.cnt[j];
            S.cnt[j] = pre.cnt;
            for (int a = 0; a < 3; ++a) {
                pre.lo[a] = min(pre.lo[a], S.blo[a][j]);
                pre.hi[a] = max(pre.hi[a], S.bhi[a][j]);
                S.blo[a][j] = pre.lo[a];
                S.bhi[a][j] = pre.hi[a];
            }
        }
        __syncthreads();
        // candidate k: left = bins 0..k, right = bins k+1..nc (BVH.cpp:192-260)
        float bc = __builtin_huge_valf();
        uint32_t bk = 0xFFFFFFFFu;
        for (int32_t k = tid; k < nc; k += T) {
            const int32_t nl = (int32_t)S.cnt[k], nr = n - nl;
            if (nl <= 1 || nr <= 1) continue;
            const float l1 = o2f(S.bhi[0][k]) - o2f(S.blo[0][k]), l2 = o2f(S.bhi[1][k]) - o2f(S.blo[1][k]),
                        l3 = o2f(S.bhi[2][k]) - o2f(S.blo[2][k]);
            const float r1 = o2f(S.shi[0][k + 1]) - o2f(S.slo[0][k + 1]),
                        r2 = o2f(S.shi[1][k + 1]) - o2f(S.slo[1][k + 1]),
                        r3 = o2f(S.shi[2][k + 1]) - o2f(S.slo[2][k + 1]);
            const float sl = l1 * l2 + l2 * l3 + l3 * l1;
            const float sr = r1 * r2 + r2 * r3 + r3 * r1;
            const float cost = sl * (float)nl + sr * (float)nr;
            const uint32_t key = ((uint32_t)axis << 16) | (uint32_t)k;
            if (cost == cost && better(cost, key, bc, bk)) {  // NaN never wins a `<`
                bc = cost;
                bk = key;
            }
        }
        S.red_cost[tid] = bc;
        S.red_key[tid] = bk;
        __syncthreads();
        for (int s = T / 2; s > 0; s >>= 1) {
            if (tid < s && better(S.red_cost[tid + s], S.red_key[tid + s], S.red_cost[tid], S.red_key[tid])) {
                S.red_cost[tid] = S.red_cost[tid + s];
                S.red_key[tid] = S.red_key[tid + s];
            }
            __syncthreads();
        }
        // strict `<` against the running minimum: earlier axes win ties
        if (tid == 0 && S.red_cost[0] < S.best_cost) {
            const uint32_t k = S.red_key[0] & 0xFFFFu;
            S.best_cost = S.red_cost[0];
            S.best_key = S.red_key[0];
            S.best_split = cand[k];
            S.best_nl = S.cnt[k];
        }
    }
    __syncthreads();
    if (S.best_key == 0xFFFFFFFFu) {  // best_axis == -1 -> leaf
        make_leaf();
        return;
    }
    const int axis = (int)(S.best_key >> 16);
    const float split = S.best_split;
    const int32_t nl = (int32_t)S.best_nl;
    // stable partition: left entries to [b, b + nl), right to [b + nl, b + n), work order kept
    int32_t left_base = 0, right_base = 0;
    for (int32_t i0 = 0; i0 < n; i0 += T) {
        const int32_t i = i0 + tid;
        const bool act = i < n;
        Ent e;
        bool isl = false;
        if (act) {
            e = in[b + i];
            isl = e.c[axis] < split;
        }
        const uint64_t ml = __ballot(act && isl), mr = __ballot(act && !isl);
        if (lane == 0) S.wave_tot[wave] = (uint32_t)__popcll(ml) | ((uint32_t)__popcll(mr) << 16);
        __syncthreads();
        int32_t wl = 0, wr = 0, tl = 0, tr = 0;
        for (int w = 0; w < T / 64; ++w) {
            const uint32_t t = S.wave_tot[w];
            if (w < wave) {
                wl += (int32_t)(t & 0xFFFFu);
                wr += (int32_t)(t >> 16);
            }
            tl += (int32_t)(t & 0xFFFFu);
            tr += (int32_t)(t >> 16);
        }
        if (act) {
            const uint64_t m = isl ? ml : mr;
            const int32_t r = (int32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            const int32_t pos = isl ? left_base + wl + r : nl + right_base + wr + r;
            out[b + pos] = e;
        }
        left_base += tl;
        right_base += tr;
        __syncthreads();
    }
    if (tid == 0) {
        const int32_t id = atomicAdd(pool_count, 2);
        PNode l{}, r{};
        l.begin = b;
        l.count = nl;
        l.level = depth + 1;
        r.begin = b + nl;
        r.count = n - nl;
        r.level = depth + 1;
        pool[id] = l;
        pool[id + 1] = r;
        nd.left = id;
        nd.right = id + 1;
    }
}

__global__ __launch_bounds__(256) void subtree_sizes(const PNode* __restrict__ pool, int32_t begin, int32_t end,
                                                     int32_t* __restrict__ size) {
    const int32_t p = begin + (int32_t)(blockIdx.x * 256 + threadIdx.x);
    if (p >= end) return;
    const PNode& nd = pool[p];
    size[p] = nd.left < 0 ? 1 : 1 + size[nd.left] + size[nd.right];
}

__global__ __launch_bounds__(256) void dfs_index(const PNode* __restrict__ pool, int32_t begin, int32_t end,
                                                 const int32_t* __restrict__ size, int32_t* __restrict__ dfs) {
    const int32_t p = begin + (int32_t)(blockIdx.x * 256 + threadIdx.x);
    if (p >= end) return;
    const PNode& nd = pool[p];
    if (nd.left < 0) return;
    dfs[nd.left] = dfs[p] + 1;
    dfs[nd.right] = dfs[p] + 1 + size[nd.left];
}

__global__ __launch_bounds__(256) void emit_nodes(const PNode* __restrict__ pool, int32_t n,
                                                  const int32_t* __restrict__ dfs, CFNode* __restrict__ out) {
    const int32_t p = (int32_t)(blockIdx.x * 256 + threadIdx.x);
    if (p >= n) return;
    const PNode& nd = pool[p];
    CFNode c;
    for (int a = 0; a < 3; ++a) {
        c.bottom[a] = nd.lo[a];
        c.top[a] = nd.hi[a];
    }
    if (nd.left < 0) {
        c.u0 = 0x80000000u | (uint32_t)nd.count;
        c.u1 = (uint32_t)nd.begin;
    } else {
        c.u0 = (uint32_t)dfs[nd.left];
        c.u1 = (uint32_t)dfs[nd.right];
    }
    out[dfs[p]] = c;
}

#define GB_CHECK(x)                                                       \
    do {                                                                  \
        hipError_t e_ = (x);                                              \
        if (e_ != hipSuccess) return std::string("gpu bvh: ") + hipGetErrorString(e_); \
    } while (0)

struct DevBuf {
    void* p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

// The level loop over entries already on the device (ents[0]).
std::string build_levels(Ent* ents0, Ent* ents1, int32_t n, int leaf_min_split, CFBvh& out,
                         hipStream_t st) {
    // a binary tree with n leaves at most has 2n - 1 nodes
    const int32_t max_nodes = 2 * n + 1;
    DevBuf pool_b, tri_b, misc_b, size_b, dfs_b, node_b;
    GB_CHECK(hipMalloc(&pool_b.p, sizeof(PNode) * (size_t)max_nodes));
    GB_CHECK(hipMalloc(&tri_b.p, sizeof(int32_t) * (size_t)n));
    GB_CHECK(hipMalloc(&misc_b.p, 64));
    PNode* pool = (PNode*)pool_b.p;
    int32_t* misc = (int32_t*)misc_b.p;  // [0] pool count, [1] flags
    PNode root{};
    root.begin = 0;
    root.count = n;
    root.level = 0;
    root.left = root.right = -1;
    GB_CHECK(hipMemcpyAsync(pool, &root, sizeof(root), hipMemcpyHostToDevice, st));
    const int32_t init[2] = {1, 0};
    GB_CHECK(hipMemcpyAsync(misc, init, sizeof(init), hipMemcpyHostToDevice, st));

    std::vector<int32_t> level_start{0, 1};
    Ent* cur = ents0;
    Ent* nxt = ents1;
    for (int level = 0;; ++level) {
        const int32_t lb = level_start[level], le = level_start[level + 1];
        if (le == lb) break;
        if (level > 4096) return "gpu bvh: runaway depth";
        // few, large nodes near the root: 512 threads each; from depth 8 on (<= 113
        // candidates per axis) one wave per node with small LDS tables
        if (level >= 8)
            split_level<64, 128><<<le - lb, 64, 0, st>>>(pool, lb, cur, nxt, (int32_t*)tri_b.p, misc,
                                                         leaf_min_split, misc + 1);
        else if (le - lb < 256)
            split_level<512, kMaxCand><<<le - lb, 512, 0, st>>>(pool, lb, cur, nxt, (int32_t*)tri_b.p, misc,
                                                                leaf_min_split, misc + 1);
        else
            split_level<256, kMaxCand><<<le - lb, 256, 0, st>>>(pool, lb, cur, nxt, (int32_t*)tri_b.p, misc,
                                                                leaf_min_split, misc + 1);
        GB_CHECK(hipGetLastError());
        int32_t h[2];
        GB_CHECK(hipMemcpyAsync(h, misc, sizeof(h), hipMemcpyDeviceToHost, st));
        GB_CHECK(hipStreamSynchronize(st));
        if (h[1]) return "gpu bvh: more split candidates than the builder holds";
        level_start.push_back(h[0]);
        Ent* t = cur;
        cur = nxt;
        nxt = t;
    }
    const int32_t total = level_start.back();
    const int levels = (int)level_start.size() - 2;  // deepest level index + 1
    GB_CHECK(hipMalloc(&size_b.p, sizeof(int32_t) * (size_t)total));
    GB_CHECK(hipMalloc(&dfs_b.p, sizeof(int32_t) * (size_t)total));
    GB_CHECK(hipMalloc(&node_b.p, sizeof(CFNode) * (size_t)total));
    int32_t* sz = (int32_t*)size_b.p;
    int32_t* dfs = (int32_t*)dfs_b.p;
    for (int l = levels - 1; l >= 0; --l) {
        const int32_t lb = level_start[l], le = level_start[l + 1];
        subtree_sizes<<<(le - lb + 255) / 256, 256, 0, st>>>(pool, lb, le, sz);
    }
    GB_CHECK(hipMemsetAsync(dfs, 0, sizeof(int32_t), st));
    for (int l = 0; l < levels; ++l) {
        const int32_t lb = level_start[l], le = level_start[l + 1];
        dfs_index<<<(le - lb + 255) / 256, 256, 0, st>>>(pool, lb, le, sz, dfs);
    }
    emit_nodes<<<(total + 255) / 256, 256, 0, st>>>(pool, total, dfs, (CFNode*)node_b.p);
    GB_CHECK(hipGetLastError());
    out.nodes.resize((size_t)total);
    out.tri_index.resize((size_t)n);
    GB_CHECK(hipMemcpyAsync(out.nodes.data(), node_b.p, sizeof(CFNode) * (size_t)total, hipMemcpyDeviceToHost,
                            st));
    GB_CHECK(hipMemcpyAsync(out.tri_index.data(), tri_b.p, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost,
                            st));
    GB_CHECK(hipStreamSynchronize(st));
    out.max_depth = levels - 1;  // PopulateCacheFriendlyBVH's depth of the deepest node
    return "";
}

bool has_neg_zero(const float* f, size_t n) {
    for (size_t i = 0; i < n; ++i)
        if (f[i] == 0.0f && signbit(f[i])) return true;
    return false;
}

}  // namespace

std::string gpu_build_cf_bvh(int device, const std::vector<v3>& vertices, const std::vector<uint32_t>& indices,
                             CFBvh& out, int leaf_min_split, double* ms) {
    const size_t nt = indices.size() / 3;
    if (nt == 0 || nt > (size_t)1 << 28) return "gpu bvh: triangle count out of range";
    if (has_neg_zero(&vertices[0].x, vertices.size() * 3))
        return "gpu bvh: -0.0 coordinates (the reference's min3/max3 tie rule is order-dependent there)";
    for (uint32_t i : indices)
        if (i >= vertices.size()) return "gpu bvh: vertex index out of range";
    GB_CHECK(hipSetDevice(device));
    const auto t0 = std::chrono::steady_clock::now();
    DevBuf v_b, i_b, e0, e1;
    GB_CHECK(hipMalloc(&v_b.p, sizeof(v3) * vertices.size()));
    GB_CHECK(hipMalloc(&i_b.p, sizeof(uint32_t) * indices.size()));
    GB_CHECK(hipMalloc(&e0.p, sizeof(Ent) * nt));
    GB_CHECK(hipMalloc(&e1.p, sizeof(Ent) * nt));
    hipStream_t st = nullptr;
    GB_CHECK(hipMemcpyAsync(v_b.p, vertices.data(), sizeof(v3) * vertices.size(), hipMemcpyHostToDevice, st));
    GB_CHECK(hipMemcpyAsync(i_b.p, indices.data(), sizeof(uint32_t) * indices.size(), hipMemcpyHostToDevice, st));
    tri_entries<<<(int)((nt + 255) / 256), 256, 0, st>>>((const float*)v_b.p, (const uint32_t*)i_b.p, (int32_t)nt,
                                                         (Ent*)e0.p);
    GB_CHECK(hipGetLastError());
    std::string err = build_levels((Ent*)e0.p, (Ent*)e1.p, (int32_t)nt, leaf_min_split, out, st);
    if (ms) *ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return err;
}

std::string gpu_build_cf_bvh_boxes(int device, const std::vector<v3>& lo, const std::vector<v3>& hi, CFBvh& out,
                                   int leaf_min_split, double* ms) {
    const size_t n = lo.size();
    if (n == 0 || n != hi.size() || n > (size_t)1 << 28) return "gpu bvh: box count out of range";
    if (has_neg_zero(&lo[0].x, n * 3) || has_neg_zero(&hi[0].x, n * 3))
        return "gpu bvh: -0.0 coordinates (the reference's min3/max3 tie rule is order-dependent there)";
    GB_CHECK(hipSetDevice(device));
    const auto t0 = std::chrono::steady_clock::now();
    DevBuf l_b, h_b, e0, e1;
    GB_CHECK(hipMalloc(&l_b.p, sizeof(v3) * n));
    GB_CHECK(hipMalloc(&h_b.p, sizeof(v3) * n));
    GB_CHECK(hipMalloc(&e0.p, sizeof(Ent) * n));
    GB_CHECK(hipMalloc(&e1.p, sizeof(Ent) * n));
    hipStream_t st = nullptr;
    GB_CHECK(hipMemcpyAsync(l_b.p, lo.data(), sizeof(v3) * n, hipMemcpyHostToDevice, st));
    GB_CHECK(hipMemcpyAsync(h_b.p, hi.data(), sizeof(v3) * n, hipMemcpyHostToDevice, st));
    box_entries<<<(int)((n + 255) / 256), 256, 0, st>>>((const float*)l_b.p, (const float*)h_b.p, (int32_t)n,
                                                        (Ent*)e0.p);
    GB_CHECK(hipGetLastError());
    std::string err = build_levels((Ent*)e0.p, (Ent*)e1.p, (int32_t)n, leaf_min_split, out, st);
    if (ms) *ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return err;
}

}  // namespace rt
