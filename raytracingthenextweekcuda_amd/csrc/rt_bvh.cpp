// rt_bvh.cpp — see rt_bvh.h. Compiled with -ffp-contract=off: the split search
// must round exactly like the reference build to reproduce its trees.
#include "rt_bvh.h"

#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <filesystem>
#include <fstream>
#include <memory>

namespace rt {

namespace {

// min3 / max3 (LinearAlgebra.h:48-49): component-wise with a strict compare.
inline v3 min3v(v3 a, v3 b) {
    return v3{a.x < b.x ? a.x : b.x, a.y < b.y ? a.y : b.y, a.z < b.z ? a.z : b.z};
}
inline v3 max3v(v3 a, v3 b) {
    return v3{a.x > b.x ? a.x : b.x, a.y > b.y ? a.y : b.y, a.z > b.z ? a.z : b.z};
}
inline float axis_of(v3 v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }

struct Entry {  // BBoxTmp (BVH.cpp:61-76)
    v3 bottom, top, center;
    int32_t tri;
};

struct BNode {
    v3 bottom{0, 0, 0}, top{0, 0, 0};
    int left = -1, right = -1;    // inner node children (pool indices)
    std::vector<int32_t> tris;    // leaf triangle list (work order)
    bool leaf() const { return left < 0; }
};

struct Builder {
    std::vector<BNode> pool;

    int make_leaf(const std::vector<Entry>& work) {
        pool.emplace_back();
        for (const Entry& e : work) pool.back().tris.push_back(e.tri);
        return (int)pool.size() - 1;
    }

    size_t leaf_min_split = 4;      // Recurse makes a leaf below 4 entries (BVH.cpp:106)

    // Split search of Recurse (BVH.cpp:136-260) in O(N log N + bins log N) per
    // axis, same result bit for bit: the left set of a candidate split is
    // {center < split}, a prefix of the entries sorted by center, so its count
    // is a lower_bound and its box a prefix reduction (the right set a
    // suffix). min3/max3 keep, among equal values, the LAST entry in work order
    // (r < v ? r : v), which only shows for -0.0 vs +0.0; the reductions below
    // break ties on work order the same way. Costs and the strict `<` argmin run
    // over the same (axis, split) sequence as the reference.
    struct Ext {
        float v;
        uint32_t w;  // work index of the entry that supplied v
    };
    static Ext take_min(Ext a, Ext b) { return a.v < b.v ? a : (b.v < a.v ? b : (a.w > b.w ? a : b)); }
    static Ext take_max(Ext a, Ext b) { return a.v > b.v ? a : (b.v > a.v ? b : (a.w > b.w ? a : b)); }
    struct Box6 {
        Ext lo[3], hi[3];
    };
    static Box6 empty_box() {
        Box6 b;
        for (int a = 0; a < 3; ++a) {
            b.lo[a] = Ext{FLT_MAX, 0};
            b.hi[a] = Ext{-FLT_MAX, 0};
        }
        return b;
    }

    void search_fast(const std::vector<Entry>& work, v3 bottom, v3 top, int depth, float& min_cost,
                     float& best_split, int& best_axis) {
        const size_t n = work.size();
        std::vector<uint32_t> order(n);
        std::vector<float> keys(n);
        std::vector<Box6> pre(n), suf(n + 1);
        for (int axis = 0; axis < 3; ++axis) {
            const float start = axis_of(bottom, axis), stop = axis_of(top, axis);
            if ((double)fabsf(stop - start) < 1e-4) continue;
            const float step = (stop - start) / (1024.0f / ((float)depth + 1.0f));
            for (size_t i = 0; i < n; ++i) order[i] = (uint32_t)i;
            std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
                const float ca = axis_of(work[a].center, axis), cb = axis_of(work[b].center, axis);
                return ca < cb || (!(cb < ca) && a < b);
            });
            Box6 acc = empty_box();
            for (size_t i = 0; i < n; ++i) {
                const Entry& e = work[order[i]];
                keys[i] = axis_of(e.center, axis);
                for (int a = 0; a < 3; ++a) {
                    acc.lo[a] = take_min(acc.lo[a], Ext{axis_of(e.bottom, a), order[i]});
                    acc.hi[a] = take_max(acc.hi[a], Ext{axis_of(e.top, a), order[i]});
                }
                pre[i] = acc;
            }
            acc = empty_box();
            suf[n] = acc;
            for (size_t i = n; i-- > 0;) {
                const Entry& e = work[order[i]];
                for (int a = 0; a < 3; ++a) {
                    acc.lo[a] = take_min(acc.lo[a], Ext{axis_of(e.bottom, a), order[i]});
                    acc.hi[a] = take_max(acc.hi[a], Ext{axis_of(e.top, a), order[i]});
                }
                suf[i] = acc;
            }
            for (float split = start + step; split < stop - step; split += step) {
                const size_t nl = (size_t)(std::lower_bound(keys.begin(), keys.begin() + n, split) -
                                           keys.begin());
                const size_t nr = n - nl;
                if (nl <= 1 || nr <= 1) continue;
                const Box6& L = pre[nl - 1];
                const Box6& R = suf[nl];
                const float l1 = L.hi[0].v - L.lo[0].v, l2 = L.hi[1].v - L.lo[1].v, l3 = L.hi[2].v - L.lo[2].v;
                const float r1 = R.hi[0].v - R.lo[0].v, r2 = R.hi[1].v - R.lo[1].v, r3 = R.hi[2].v - R.lo[2].v;
                const float sl = l1 * l2 + l2 * l3 + l3 * l1;
                const float sr = r1 * r2 + r2 * r3 + r3 * r1;
                const float cost = sl * (float)(int)nl + sr * (float)(int)nr;
                if (cost < min_cost) {
                    min_cost = cost;
                    best_split = split;
                    best_axis = axis;
                }
            }
        }
    }

    // Recurse (BVH.cpp:94-333).
    int recurse(std::vector<Entry>& work, int depth) {
        if (work.size() < leaf_min_split) return make_leaf(work);

        v3 bottom{FLT_MAX, FLT_MAX, FLT_MAX}, top{-FLT_MAX, -FLT_MAX, -FLT_MAX};
        for (const Entry& v : work) {
            bottom = min3v(bottom, v.bottom);
            top = max3v(top, v.top);
        }
        const float side1 = top.x - bottom.x, side2 = top.y - bottom.y, side3 = top.z - bottom.z;
        float min_cost = (float)work.size() * (side1 * side2 + side2 * side3 + side3 * side1);
        float best_split = FLT_MAX;
        int best_axis = -1;

        // (the reference's O(N x bins) loop, BVH.cpp:160-260, is restated in the oracle,
        // oracle/rt_oracle.c orc_bvh_image, which tests/test_bvh.py compares with this search)
        search_fast(work, bottom, top, depth, min_cost, best_split, best_axis);
        if (best_axis == -1) return make_leaf(work);

        std::vector<Entry> left, right;
        v3 lb{FLT_MAX, FLT_MAX, FLT_MAX}, lt{-FLT_MAX, -FLT_MAX, -FLT_MAX};
        v3 rb{FLT_MAX, FLT_MAX, FLT_MAX}, rtp{-FLT_MAX, -FLT_MAX, -FLT_MAX};
        for (const Entry& v : work) {
            if (axis_of(v.center, best_axis) < best_split) {
                left.push_back(v);
                lb = min3v(lb, v.bottom);
                lt = max3v(lt, v.top);
            } else {
                right.push_back(v);
                rb = min3v(rb, v.bottom);
                rtp = max3v(rtp, v.top);
            }
        }
        work.clear();
        work.shrink_to_fit();
        pool.emplace_back();
        const int me = (int)pool.size() - 1;
        const int l = recurse(left, depth + 1);
        pool[l].bottom = lb;
        pool[l].top = lt;
        const int r = recurse(right, depth + 1);
        pool[r].bottom = rb;
        pool[r].top = rtp;
        pool[me].left = l;
        pool[me].right = r;
        return me;
    }

    // PopulateCacheFriendlyBVH (BVH.cpp:432-465): depth first, left first.
    void populate(int n, uint32_t& idx_boxes, CFBvh& out, int depth) {
        if (depth > out.max_depth) out.max_depth = depth;
        const uint32_t cur = idx_boxes;
        CFNode& c = out.nodes[cur];
        const BNode& b = pool[n];
        c.bottom[0] = b.bottom.x; c.bottom[1] = b.bottom.y; c.bottom[2] = b.bottom.z;
        c.top[0] = b.top.x; c.top[1] = b.top.y; c.top[2] = b.top.z;
        if (!b.leaf()) {
            const uint32_t il = ++idx_boxes;
            populate(b.left, idx_boxes, out, depth + 1);
            const uint32_t ir = ++idx_boxes;
            populate(b.right, idx_boxes, out, depth + 1);
            out.nodes[cur].u0 = il;
            out.nodes[cur].u1 = ir;
        } else {
            out.nodes[cur].u0 = 0x80000000u | (uint32_t)b.tris.size();
            out.nodes[cur].u1 = (uint32_t)out.tri_index.size();
            for (int32_t t : b.tris) out.tri_index.push_back(t);
        }
    }
};

}  // namespace

std::string load_ply(const std::string& path, PlyMesh& out) {
    std::ifstream in(path);
    if (!in) return "cannot open PLY file: " + path;
    out.vertices.clear();
    out.indices.clear();
    std::string line;
    unsigned nv = 0, nf = 0;
    bool inside = false;
    while (std::getline(in, line)) {
        if (!inside) {
            if (line.compare(0, 14, "element vertex") == 0) {
                nv = (unsigned)strtoul(line.c_str() + 14, nullptr, 10);
            } else if (line.compare(0, 12, "element face") == 0) {
                nf = (unsigned)strtoul(line.c_str() + 12, nullptr, 10);
            } else if (line.compare(0, 10, "end_header") == 0) {
                inside = true;
                // header counts are untrusted: reserve at most 16M entries up front
                out.vertices.reserve(std::min<size_t>(nv, (size_t)1 << 24));
                out.indices.reserve(std::min<size_t>((size_t)nf * 3, (size_t)3 << 24));
            }
        } else if (nv) {
            --nv;
            // str_in >> x >> y >> z (Loader.cpp:258-259): correctly rounded strtof.
            const char* p = line.c_str();
            char* e;
            float x = strtof(p, &e);
            float y = strtof(e, &e);
            float z = strtof(e, &e);
            out.vertices.push_back(v3{x, y, z});
        } else if (nf) {
            --nf;
            // `dummy idx1 idx2 idx3` (Loader.cpp:276-277): only the first three
            // indices of a face are used.
            unsigned long v[4];
            const char* p = line.c_str();
            char* e;
            int k = 0;
            for (; k < 4; ++k) {
                v[k] = strtoul(p, &e, 10);
                if (e == p) break;
                p = e;
            }
            if (k < 4) continue;  // malformed line: skipped like a failed `>>`
            const size_t n = out.vertices.size();
            if (v[1] >= n || v[2] >= n || v[3] >= n) return "PLY face index out of range in " + path;
            out.indices.push_back((uint32_t)v[1]);
            out.indices.push_back((uint32_t)v[2]);
            out.indices.push_back((uint32_t)v[3]);
        }
    }
    if (!inside) return "PLY header without end_header: " + path;
    return "";
}

void process_ply_vertices(PlyMesh& m, v3 offset, float max_coord) {
    v3 minp{FLT_MAX, FLT_MAX, FLT_MAX}, maxp{-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (size_t i = 0; i < m.indices.size(); i += 3) {
        for (int k = 0; k < 3; ++k) minp = min3v(minp, m.vertices[m.indices[i + k]]);
        for (int k = 0; k < 3; ++k) maxp = max3v(maxp, m.vertices[m.indices[i + k]]);
    }
    const v3 c{(maxp.x + minp.x) * 0.5f, (maxp.y + minp.y) * 0.5f, (maxp.z + minp.z) * 0.5f};
    minp = sub(minp, c);
    maxp = sub(maxp, c);
    float maxi = 0.0f;  // std::max(maxi, (float)fabs(.)) keeps the first on ties
    const float cand[6] = {fabsf(minp.x), fabsf(minp.y), fabsf(minp.z),
                           fabsf(maxp.x), fabsf(maxp.y), fabsf(maxp.z)};
    for (float f : cand) maxi = (maxi < f) ? f : maxi;
    const float s = max_coord / maxi;
    for (v3& v : m.vertices) {
        v = sub(v, c);
        v = scale(v, s);
        v = add(v, offset);
    }
}

void build_cf_bvh_boxes(const std::vector<v3>& bottoms, const std::vector<v3>& tops, CFBvh& out,
                        int leaf_min_split) {
    // CreateBVH (BVH.cpp:335-392) over precomputed primitive boxes.
    const size_t nt = bottoms.size();
    std::vector<Entry> work;
    work.reserve(nt);
    v3 bottom{FLT_MAX, FLT_MAX, FLT_MAX}, top{-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (size_t j = 0; j < nt; ++j) {
        Entry b;
        b.tri = (int32_t)j;
        b.bottom = bottoms[j];
        b.top = tops[j];
        bottom = min3v(bottom, b.bottom);
        top = max3v(top, b.top);
        b.center = scale(add(b.top, b.bottom), 0.5f);
        work.push_back(b);
    }
    Builder B;
    B.leaf_min_split = (size_t)leaf_min_split;
    B.pool.reserve(nt);
    const int root = B.recurse(work, 0);
    B.pool[root].bottom = bottom;
    B.pool[root].top = top;
    // CreateCFBVH (BVH.cpp:467-497).
    out.nodes.assign(B.pool.size(), CFNode{});
    out.tri_index.clear();
    out.tri_index.reserve(nt);
    out.max_depth = 0;
    uint32_t idx = 0;
    B.populate(root, idx, out, 0);
}

void build_cf_bvh(const std::vector<v3>& vertices, const std::vector<uint32_t>& indices,
                  CFBvh& out, int leaf_min_split) {
    // Per-triangle boxes: min3/max3 over the three vertices from FLT_MAX seeds.
    const size_t nt = indices.size() / 3;
    std::vector<v3> lo(nt), hi(nt);
    for (size_t j = 0; j < nt; ++j) {
        v3 b{FLT_MAX, FLT_MAX, FLT_MAX}, t{-FLT_MAX, -FLT_MAX, -FLT_MAX};
        for (int k = 0; k < 3; ++k) b = min3v(b, vertices[indices[3 * j + k]]);
        for (int k = 0; k < 3; ++k) t = max3v(t, vertices[indices[3 * j + k]]);
        lo[j] = b;
        hi[j] = t;
    }
    build_cf_bvh_boxes(lo, hi, out, leaf_min_split);
}

namespace {
inline float vlen(v3 a) { return sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); }
// Vector3Df::normalize (LinearAlgebra.h:30): in place, x /= norm ...
inline v3 vnormalize(v3 a) {
    const float n = sqrtf(a.x * a.x + a.y * a.y + a.z * a.z);
    return v3{a.x / n, a.y / n, a.z / n};
}
}  // namespace

void kuchkuda_triangles(const PlyMesh& m, const std::vector<uint32_t>& materials,
                        std::vector<KTri>& out) {
    const size_t nt = m.indices.size() / 3;
    out.resize(nt);
    for (size_t i = 0; i < nt; ++i) {
        const v3 a = m.vertices[m.indices[3 * i]], b = m.vertices[m.indices[3 * i + 1]],
                 c = m.vertices[m.indices[3 * i + 2]];
        const v3 vc1 = sub(b, a), vc2 = sub(c, b), vc3 = sub(a, c);
        v3 n = cross(vc1, vc2);
        const v3 alt1 = cross(vc2, vc3);
        if (vlen(alt1) > vlen(n)) n = alt1;
        const v3 alt2 = cross(vc3, vc1);
        if (vlen(alt2) > vlen(n)) n = alt2;
        n = vnormalize(n);
        const v3 e1 = vnormalize(cross(n, vc1)), e2 = vnormalize(cross(n, vc2)),
                 e3 = vnormalize(cross(n, vc3));
        KTri& t = out[i];
        t.n[0] = n.x; t.n[1] = n.y; t.n[2] = n.z; t.d = dot(n, a);
        t.e1[0] = e1.x; t.e1[1] = e1.y; t.e1[2] = e1.z; t.d1 = dot(e1, a);
        t.e2[0] = e2.x; t.e2[1] = e2.y; t.e2[2] = e2.z; t.d2 = dot(e2, b);
        t.e3[0] = e3.x; t.e3[1] = e3.y; t.e3[2] = e3.z; t.d3 = dot(e3, c);
        t.material = (float)materials[i];
        t.pad[0] = t.pad[1] = t.pad[2] = 0.0f;
    }
}

std::string append_ply(const std::string& path, PlyMesh& accum) {
    PlyMesh m;
    std::string e = load_ply(path, m);
    if (!e.empty()) return e;
    const uint32_t base = (uint32_t)accum.vertices.size();
    accum.vertices.insert(accum.vertices.end(), m.vertices.begin(), m.vertices.end());
    for (uint32_t i : m.indices) accum.indices.push_back(i + base);
    return "";
}

std::vector<uint8_t> bvh_image(const CFBvh& b) {
    const uint32_t nn = (uint32_t)b.nodes.size(), ni = (uint32_t)b.tri_index.size();
    std::vector<uint8_t> img(8 + (size_t)nn * sizeof(CFNode) + (size_t)ni * 4);
    memcpy(img.data(), &nn, 4);
    memcpy(img.data() + 4, &ni, 4);
    memcpy(img.data() + 8, b.nodes.data(), (size_t)nn * sizeof(CFNode));
    memcpy(img.data() + 8 + (size_t)nn * sizeof(CFNode), b.tri_index.data(), (size_t)ni * 4);
    return img;
}

std::string parse_bvh_image(const uint8_t* data, size_t size, const std::vector<v3>& vertices,
                            const std::vector<uint32_t>& indices, CFBvh& out) {
    if (!data || size < 8) return "shorter than its 8-byte header";
    uint32_t nn = 0, ni = 0;
    memcpy(&nn, data, 4);
    memcpy(&ni, data + 4, 4);
    const size_t nt = indices.size() / 3;
    if (nn == 0) return "no nodes";
    if ((uint64_t)ni != (uint64_t)nt) return "index count does not match the triangle count";
    if ((uint64_t)size != 8ull + 32ull * nn + 4ull * ni) return "size does not match the header counts";
    CFBvh b;
    b.nodes.resize(nn);
    b.tri_index.resize(ni);
    memcpy(b.nodes.data(), data + 8, (size_t)nn * sizeof(CFNode));
    memcpy(b.tri_index.data(), data + 8 + (size_t)nn * sizeof(CFNode), (size_t)ni * 4);
    std::vector<uint8_t> seen(nt, 0), covered(ni, 0), parents(nn, 0);
    for (uint32_t k = 0; k < ni; ++k) {
        const int32_t t = b.tri_index[k];
        if (t < 0 || (size_t)t >= nt) return "triangle index out of range";
        if (seen[(size_t)t]++) return "triangle listed twice";
    }
    std::vector<int> depth(nn, 0);
    for (uint32_t i = 0; i < nn; ++i) {
        const CFNode& n = b.nodes[i];
        for (int a = 0; a < 3; ++a)
            if (!std::isfinite(n.bottom[a]) || !std::isfinite(n.top[a]) || n.bottom[a] > n.top[a])
                return "bad box at node " + std::to_string(i);
        if (i > 0 && parents[i] != 1) return "node " + std::to_string(i) + " is not referenced exactly once";
        if (depth[i] > b.max_depth) b.max_depth = depth[i];
        auto inside = [&](const float* lo, const float* hi, v3 p) {
            return p.x >= lo[0] && p.x <= hi[0] && p.y >= lo[1] && p.y <= hi[1] && p.z >= lo[2] && p.z <= hi[2];
        };
        if (n.u0 & 0x80000000u) {
            const uint32_t cnt = n.u0 & 0x7FFFFFFFu, st = n.u1;
            if (cnt == 0 || (uint64_t)st + cnt > ni) return "leaf range out of bounds at node " + std::to_string(i);
            for (uint32_t k = st; k < st + cnt; ++k) {
                if (covered[k]++) return "leaves overlap in the triangle list";
                const size_t t = (size_t)b.tri_index[k];
                for (int j = 0; j < 3; ++j)
                    if (!inside(n.bottom, n.top, vertices[indices[3 * t + (size_t)j]]))
                        return "leaf box does not contain its triangles at node " + std::to_string(i);
            }
        } else {
            const uint32_t l = n.u0, r = n.u1;
            if (l <= i || r <= i || l >= nn || r >= nn || l == r) return "bad children at node " + std::to_string(i);
            for (uint32_t ch : {l, r}) {
                const CFNode& cn = b.nodes[ch];
                if (!inside(n.bottom, n.top, v3{cn.bottom[0], cn.bottom[1], cn.bottom[2]}) ||
                    !inside(n.bottom, n.top, v3{cn.top[0], cn.top[1], cn.top[2]}))
                    return "child box outside its parent at node " + std::to_string(i);
                ++parents[ch];
                depth[ch] = depth[i] + 1;
            }
        }
    }
    for (uint32_t k = 0; k < ni; ++k)
        if (!covered[k]) return "triangle list entry not in any leaf";
    out = std::move(b);
    return "";
}

int read_bvh_cache(const std::string& ply_path, const std::vector<v3>& vertices, const std::vector<uint32_t>& indices,
                   CFBvh& out, std::string* why) {
    namespace fs = std::filesystem;
    const std::string cache = ply_path + ".bvh";
    std::error_code ec;
    if (!fs::exists(cache, ec) || ec) return 0;
    if (fs::exists(ply_path, ec) && !ec) {
        const auto tp = fs::last_write_time(ply_path, ec);
        const auto tb = ec ? tp : fs::last_write_time(cache, ec);
        if (!ec && tp > tb) return 0;  // bUpdateBVH = plyFileTime > bvhFileTime (BVH.cpp:508-514)
    }
    FILE* fp = fopen(cache.c_str(), "rb");
    if (!fp) return 0;
    std::vector<uint8_t> img;
    uint8_t buf[1 << 16];
    size_t got;
    while ((got = fread(buf, 1, sizeof(buf), fp)) > 0) {
        img.insert(img.end(), buf, buf + got);
        if (img.size() > ((size_t)1 << 33)) break;  // > 8 GiB: not a cache of any loadable mesh
    }
    fclose(fp);
    const std::string e = parse_bvh_image(img.data(), img.size(), vertices, indices, out);
    if (!e.empty()) {
        if (why) *why = cache + ": " + e;
        return -1;
    }
    return 1;
}

bool write_bvh_cache(const std::string& ply_path, const CFBvh& b) {
    const std::vector<uint8_t> img = bvh_image(b);
    FILE* fp = fopen((ply_path + ".bvh").c_str(), "wb");
    if (!fp) return false;
    const bool ok = fwrite(img.data(), 1, img.size(), fp) == img.size();
    return fclose(fp) == 0 && ok;
}

namespace {
struct CFPairBuilder {
    std::vector<CFNode>& nodes;
    int max_pairs = 0;
    bool empty_leaf = false;

    uint32_t alloc() {
        const size_t at = nodes.size();
        nodes.resize(at + 2, CFNode{});
        return (uint32_t)(at / 2);
    }
    void set(uint32_t q, CFNode l, uint32_t ref_l, uint32_t leaf_l, CFNode r, uint32_t ref_r, uint32_t leaf_r) {
        l.u0 = ref_l;
        l.u1 = leaf_l;
        r.u0 = ref_r;
        r.u1 = leaf_r;
        nodes[2 * (size_t)q] = l;
        nodes[2 * (size_t)q + 1] = r;
    }
    uint32_t leaf(CFNode box, uint32_t first, uint32_t count, int above) {
        if (count <= kLeafRefMax) {
            empty_leaf |= count == 0u;
            max_pairs = std::max(max_pairs, above);
            return kLeafRef | ((count - 1u) << 27) | first;
        }
        const uint32_t q = alloc();  // a larger leaf: two halves under the leaf's box
        const uint32_t half = count / 2u;
        const uint32_t l = leaf(box, first, half, above + 1), r = leaf(box, first + half, count - half, above + 1);
        set(q, box, l, 1u, box, r, 1u);
        return q;
    }
    uint32_t node(uint32_t i, int above) {
        const CFNode n = nodes[i];
        if (n.u0 & 0x80000000u) return leaf(n, n.u1, n.u0 & 0x7FFFFFFFu, above);
        const uint32_t q = alloc();
        const uint32_t l = node(n.u0, above + 1), r = node(n.u1, above + 1);
        const CFNode a = nodes[n.u0], b = nodes[n.u1];
        set(q, a, l, (a.u0 >> 31), b, r, (b.u0 >> 31));
        return q;
    }
};
}  // namespace

uint32_t cf_child_pairs(std::vector<CFNode>& nodes, int* max_pairs, bool* empty_leaf) {
    *max_pairs = 0;
    *empty_leaf = false;
    if (nodes.empty()) return 0;
    if (nodes.size() & 1u) nodes.push_back(CFNode{});
    CFPairBuilder pb{nodes};
    const uint32_t root = pb.node(0, 0);
    *max_pairs = pb.max_pairs;
    *empty_leaf = pb.empty_leaf;
    return root;
}

}  // namespace rt
