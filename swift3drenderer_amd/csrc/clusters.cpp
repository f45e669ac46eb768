// clusters.cpp -- init-time spatial clusters of the triangle list (tile path, render_api.cpp).
//
// render.cpp:297 visits every triangle every frame; so does the tile path's per-triangle setup, on
// every GPU of a row-band split, although a GPU owns only 1/N of the rows.  Grouping the triangles
// once, at load time, into small spatially compact clusters with a bounding sphere lets a per-frame
// kernel (kernels.hip k_cluster_cull) reject a whole cluster -- behind the near plane, off screen, or
// outside this GPU's rows -- with one test, so the setup reads only the triangles that can reach the
// part.  The tile path is order-independent (per pixel the max (1/z, ~slot) key wins), so the order
// in which clusters and their triangles are set up does not change a pixel; every triangle keeps its
// slot id for the tie order.
//
// Clusters: the connected components of the index graph (triangles sharing a vertex index are one
// mesh: an icosahedron of the stress scene is one 20-triangle component), taken whole when they
// hold kMin..kMax triangles; larger ones are cut into kMax-triangle pieces along the Morton order of
// their triangle centroids; smaller ones (loose triangles, tiny meshes) are pooled, sorted by the
// Morton code of their centroids over the scene's box and packed into clusters of up to kMax.
// Plain C++ (g++): runs once per scene load.
#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <numeric>
#include <vector>

namespace s3r_host {

namespace {

uint32_t find_root(std::vector<uint32_t> &par, uint32_t v) {
    while (par[v] != v) {
        par[v] = par[par[v]];                         // path halving
        v = par[v];
    }
    return v;
}

// 3 x 21-bit Morton code of a point already scaled into [0, 2^21)
uint64_t spread21(uint64_t x) {
    x &= 0x1FFFFFull;
    x = (x | x << 32) & 0x1F00000000FFFFull;
    x = (x | x << 16) & 0x1F0000FF0000FFull;
    x = (x | x << 8) & 0x100F00F00F00F00Full;
    x = (x | x << 4) & 0x10C30C30C30C30C3ull;
    x = (x | x << 2) & 0x1249249249249249ull;
    return x;
}

struct Box {
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    void add(const float *p) {
        for (int k = 0; k < 3; k++) {
            lo[k] = std::min(lo[k], (double)p[k]);
            hi[k] = std::max(hi[k], (double)p[k]);
        }
    }
};

uint64_t morton(const Box &b, const double c[3]) {
    uint64_t code = 0;
    for (int k = 0; k < 3; k++) {
        const double ext = b.hi[k] - b.lo[k];
        double u = ext > 0 ? (c[k] - b.lo[k]) / ext : 0.0;
        if (!std::isfinite(u)) u = 0.0;                       // (a non-finite vertex)
        u = std::min(std::max(u, 0.0), 1.0) * 2097151.0;
        code |= spread21((uint64_t)u) << k;
    }
    return code;
}

}  // namespace

// vtx: nv x float4 (x, y, z, w); vidx: 3 ntri vertex indices (< nv, checked by the reader).
// Output: first (C + 1 position ranges), sphere (4 C floats: centre, radius -- +inf for a cluster
// with a non-finite vertex, which the cull never rejects), perm (position -> triangle; left empty
// when it is the identity).
void build_clusters(const float *vtx, uint32_t nv, const uint32_t *vidx, uint32_t ntri, uint32_t kmin, uint32_t kmax,
                    std::vector<uint32_t> &first, std::vector<float> &sphere, std::vector<uint32_t> &perm) {
    first.assign(1, 0u);
    sphere.clear();
    perm.clear();
    if (ntri == 0) return;
    // connected components of the index graph
    std::vector<uint32_t> par(nv);
    std::iota(par.begin(), par.end(), 0u);
    for (uint32_t t = 0; t < ntri; t++) {
        const uint32_t a = find_root(par, vidx[3 * t]);
        for (int k = 1; k < 3; k++) {
            const uint32_t b = find_root(par, vidx[3 * t + k]);
            if (a != b) par[std::max(a, b)] = std::min(a, b);
        }
    }
    // component ids in order of first appearance
    std::vector<uint32_t> comp_id(nv, 0xFFFFFFFFu), comp(ntri), csize;
    for (uint32_t t = 0; t < ntri; t++) {
        uint32_t &id = comp_id[find_root(par, vidx[3 * t])];
        if (id == 0xFFFFFFFFu) {
            id = (uint32_t)csize.size();
            csize.push_back(0);
        }
        comp[t] = id;
        csize[id]++;
    }
    std::vector<uint32_t>().swap(par);
    std::vector<uint32_t>().swap(comp_id);
    const uint32_t ncomp = (uint32_t)csize.size();
    // triangles grouped by component (stable: file order inside a component)
    std::vector<uint64_t> cstart(ncomp + 1, 0);
    for (uint32_t c = 0; c < ncomp; c++) cstart[c + 1] = cstart[c] + csize[c];
    std::vector<uint32_t> order(ntri);
    {
        std::vector<uint64_t> cur(cstart.begin(), cstart.end() - 1);
        for (uint32_t t = 0; t < ntri; t++) order[cur[comp[t]]++] = t;
    }
    std::vector<uint32_t>().swap(comp);
    auto centroid = [&](uint32_t t, double c[3]) {
        for (int k = 0; k < 3; k++)
            c[k] = ((double)vtx[4 * vidx[3 * t] + k] + vtx[4 * vidx[3 * t + 1] + k] + vtx[4 * vidx[3 * t + 2] + k]) / 3.0;
    };
    Box scene;
    for (uint32_t v = 0; v < nv; v++)
        if (std::isfinite(vtx[4 * v]) && std::isfinite(vtx[4 * v + 1]) && std::isfinite(vtx[4 * v + 2])) scene.add(vtx + 4 * v);

    perm.reserve(ntri);
    auto emit = [&](const uint32_t *tris, uint32_t n) {           // one cluster
        perm.insert(perm.end(), tris, tris + n);
        first.push_back((uint32_t)perm.size());
    };
    std::vector<std::pair<uint64_t, uint32_t>> keyed;
    std::vector<uint32_t> tmp;
    std::vector<std::pair<uint64_t, uint32_t>> pool;           // (Morton code, component) of small components
    for (uint32_t c = 0; c < ncomp; c++) {
        const uint32_t *tris = order.data() + cstart[c];
        const uint32_t n = csize[c];
        if (n >= kmin && n <= kmax) {
            emit(tris, n);
        } else if (n > kmax) {                                  // cut along the Morton order of centroids
            Box b;
            for (uint32_t i = 0; i < n; i++)
                for (int k = 0; k < 3; k++) b.add(vtx + 4 * vidx[3 * tris[i] + k]);
            keyed.resize(n);
            for (uint32_t i = 0; i < n; i++) {
                double ct[3];
                centroid(tris[i], ct);
                keyed[i] = {morton(b, ct), tris[i]};
            }
            std::sort(keyed.begin(), keyed.end());
            tmp.resize(n);
            for (uint32_t i = 0; i < n; i++) tmp[i] = keyed[i].second;
            const uint32_t pieces = (n + kmax - 1) / kmax;
            for (uint32_t q = 0; q < pieces; q++) {
                const uint32_t a = (uint32_t)((uint64_t)n * q / pieces), e = (uint32_t)((uint64_t)n * (q + 1) / pieces);
                emit(tmp.data() + a, e - a);
            }
        } else {
            double ct[3] = {0, 0, 0};
            for (uint32_t i = 0; i < n; i++) {
                double tc[3];
                centroid(tris[i], tc);
                for (int k = 0; k < 3; k++) ct[k] += tc[k] / n;
            }
            pool.push_back({morton(scene, ct), c});
        }
    }
    // small components: packed along the Morton order of their centroids
    std::sort(pool.begin(), pool.end());
    tmp.clear();
    for (const auto &pc : pool) {
        const uint32_t c = pc.second, n = csize[c];
        if (!tmp.empty() && tmp.size() + n > kmax) {
            emit(tmp.data(), (uint32_t)tmp.size());
            tmp.clear();
        }
        tmp.insert(tmp.end(), order.data() + cstart[c], order.data() + cstart[c] + n);
    }
    if (!tmp.empty()) emit(tmp.data(), (uint32_t)tmp.size());

    // bounding spheres: the centre of the cluster's vertex box (rounded to float), the radius the
    // largest distance from that float centre, in double, rounded up with a relative margin
    const uint32_t ncl = (uint32_t)first.size() - 1;
    sphere.resize(4 * (size_t)ncl);
    for (uint32_t q = 0; q < ncl; q++) {
        Box b;
        bool finite = true;
        for (uint32_t i = first[q]; i < first[q + 1]; i++)
            for (int k = 0; k < 3; k++) {
                const float *p = vtx + 4 * vidx[3 * perm[i] + k];
                finite = finite && std::isfinite(p[0]) && std::isfinite(p[1]) && std::isfinite(p[2]);
                b.add(p);
            }
        float ctr[3];
        for (int k = 0; k < 3; k++) ctr[k] = finite ? (float)((b.lo[k] + b.hi[k]) * 0.5) : 0.0f;
        double r2 = 0;
        for (uint32_t i = first[q]; i < first[q + 1] && finite; i++)
            for (int k = 0; k < 3; k++) {
                const float *p = vtx + 4 * vidx[3 * perm[i] + k];
                double d2 = 0;
                for (int a = 0; a < 3; a++) d2 += ((double)p[a] - ctr[a]) * ((double)p[a] - ctr[a]);
                r2 = std::max(r2, d2);
            }
        const double r = sqrt(r2) * (1.0 + 1e-6) + 1e-30;
        float rf = (float)r;
        if ((double)rf < r) rf = nextafterf(rf, INFINITY);
        sphere[4 * q] = ctr[0];
        sphere[4 * q + 1] = ctr[1];
        sphere[4 * q + 2] = ctr[2];
        sphere[4 * q + 3] = finite && std::isfinite(rf) ? rf : INFINITY;
    }
    bool identity = true;
    for (uint32_t i = 0; i < ntri && identity; i++) identity = perm[i] == i;
    if (identity) std::vector<uint32_t>().swap(perm);
}

}  // namespace s3r_host

// Test hook (include/render.h s3r_build_clusters): the clusters of a vertex / index list, without a
// GPU.  Returns the cluster count C; writes min(C + 1, first_cap) range starts, min(C, first_cap)
// spheres and, when perm_out is not null, ntri positions (the identity when no permutation).
extern "C" __attribute__((visibility("default"))) uint32_t s3r_build_clusters(const float *vtx, uint32_t nv,
                                                                              const uint32_t *vidx, uint32_t ntri,
                                                                              uint32_t *first_out, float *sphere_out,
                                                                              uint32_t first_cap, uint32_t *perm_out) {
    std::vector<uint32_t> first, perm;
    std::vector<float> sphere;
    s3r_host::build_clusters(vtx, nv, vidx, ntri, 8, 32, first, sphere, perm);
    const uint32_t ncl = (uint32_t)first.size() - 1;
    for (uint32_t i = 0; i < first.size() && i < first_cap; i++) first_out[i] = first[i];
    for (uint32_t i = 0; i < ncl && i < first_cap; i++)
        for (int k = 0; k < 4; k++) sphere_out[4 * i + k] = sphere[4 * i + k];
    if (perm_out)
        for (uint32_t i = 0; i < ntri; i++) perm_out[i] = perm.empty() ? i : perm[i];
    return ncl;
}
