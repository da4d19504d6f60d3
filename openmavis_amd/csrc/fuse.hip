// LocalMapping::SearchInNeighbors' fuse sequence (src/LocalMapping.cc:837-889) over ORBmatcher::Fuse
// (src/ORBmatcher.cc:1458-1647) and the map mutations it makes between its decisions (MapPoint::Replace / AddObservation
// / ComputeDistinctiveDescriptors, src/MapPoint.cc:199-226, :316-380, :405-483; KeyFrame::AddMapPoint /
// ReplaceMapPointMatch / EraseMapPointMatch).
//
// The window searches (projection, image / distance / viewing tests, KeyFrame::GetFeaturesInArea, the reprojection gate,
// the Hamming scan) are the compute: all (Fuse call, point) entries of a phase are evaluated on the device in ONE
// omv_matcher_search_kf launch, speculatively, with the descriptors as they stand.  The decisions are a sequential walk
// over a mutable graph (std::map observations, pointer-identity claims), so they run here on the host in the reference's
// order against the flattened snapshot.  An entry is valid as long as its point's descriptor is the one it was evaluated
// with: the only state a window search reads that the walk changes is GetDescriptor() -- a Replace survivor's
// ComputeDistinctiveDescriptors -- while isBad / IsInKeyFrame / GetMapPoint / Observations are read by the walk itself.
// Before each Fuse call the stale entries of the rest of the phase are re-evaluated together (one device round trip:
// the recomputed descriptors first, by the distinctive-descriptor kernel over the observation rows the reference reads
// at the Replace, then the searches); a point that goes stale inside a call (it appears again later in the same list)
// is re-evaluated when the walk reaches it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <map>
#include <vector>

#include "../../include/omv.h"
#include "omv_device.h"

#define HIP_OK(x)                                          \
    do {                                                   \
        if ((x) != hipSuccess) return OMV_ERR_HIP;         \
    } while (0)
#define OMV_OK_OR_RETURN(x)                                \
    do {                                                   \
        const omv_status s_ = (x);                         \
        if (s_ != OMV_OK) return s_;                       \
    } while (0)

namespace {

constexpr int kThLow = 50;

// mDescriptor = vDescriptors[BestIdx] of the recomputed points, into the map-point table
__global__ void fuse_desc_scatter_kernel(int n, const int32_t *mp, const int32_t *best_row, const uint8_t *desc,
                                         uint8_t *table) {
    const int k = blockIdx.x * 4 + (threadIdx.x >> 3), lane = threadIdx.x & 7;
    if (k >= n) return;
    const int r = best_row[k];
    if (r < 0) return;
    reinterpret_cast<uint32_t *>(table + (size_t)mp[k] * 32)[lane] = reinterpret_cast<const uint32_t *>(desc + (size_t)r * 32)[lane];
}

struct Obs {
    int kf;
    int idx[4];
};

struct Entry {
    int job, mp, ver;
    int best_idx, best_dist;
};

struct Walk {
    omv_matcher *m;
    const omv_frame_geom *geom;
    const omv_kp *kps;
    const uint8_t *desc;
    const int *n_kp_dev;
    int kp_cap, C, n_kf;
    omv_fuse_graph *g;
    const omv_kf_mps *mps;
    omv_kf_search_params p;
    hipStream_t st;
    std::vector<int> nkp;                   // [n_kf][C]
    std::vector<std::vector<Obs>> obs;      // per point, keyframe order
    std::vector<int> ver;                   // descriptor version per point
    std::map<int, std::vector<int>> pending;   // point -> device descriptor rows of its last ComputeDistinctiveDescriptors
    int n_log = 0, n_re = 0, n_calls = 0;
    bool overflow = false;
    // device scratch
    int32_t *d_i32 = nullptr;
    size_t d_cap = 0;

    int *kfmp(int kf) { return g->kf_mps + (size_t)kf * C * kp_cap; }
    int n_of(int kf) const {
        int n = 0;
        for (int c = 0; c < C; ++c) n += nkp[(size_t)kf * C + c];
        return n;
    }
    // the tuple slot of N-index idx (MapPoint::AddObservation, MapPoint.cc:209-218)
    int slot_of(int kf, int idx) const {
        if (g->n_blocks[kf] == 1) return 0;
        int off = 0;
        for (int c = 0; c < 3; ++c) {
            off += c < C ? nkp[(size_t)kf * C + c] : 0;
            if (idx < off) return c;
        }
        return 3;
    }
    // N-index -> row of the batch's descriptor array
    size_t row_of(int kf, int idx) const {
        int c = 0, off = 0;
        while (c + 1 < C && idx >= off + nkp[(size_t)kf * C + c]) off += nkp[(size_t)kf * C + c], ++c;
        return ((size_t)kf * C + c) * kp_cap + (idx - off);
    }
    Obs *find(int mp, int kf) {
        auto &v = obs[mp];
        auto it = std::lower_bound(v.begin(), v.end(), kf, [](const Obs &o, int k) { return o.kf < k; });
        return (it != v.end() && it->kf == kf) ? &*it : nullptr;
    }
    bool in_kf(int mp, int kf) { return find(mp, kf) != nullptr; }
    void log(int a, int b, int c, int d) {
        if (n_log < g->log_cap && g->log) {
            int32_t *r = g->log + 4 * (size_t)n_log;
            r[0] = a, r[1] = b, r[2] = c, r[3] = d;
        } else {
            overflow = true;
        }
        ++n_log;
    }
    void add_observation(int mp, int kf, int idx) {   // MapPoint::AddObservation (MapPoint.cc:199-226)
        auto &v = obs[mp];
        auto it = std::lower_bound(v.begin(), v.end(), kf, [](const Obs &o, int k) { return o.kf < k; });
        if (it == v.end() || it->kf != kf) it = v.insert(it, Obs{kf, {-1, -1, -1, -1}});
        it->idx[slot_of(kf, idx)] = idx;
        const bool stereo = g->n_blocks[kf] == 1 && g->uright && g->uright[(size_t)kf * kp_cap + idx] >= 0;
        g->n_obs[mp] += stereo ? 2 : 1;
    }
    void compute_distinctive(int mp) {   // MapPoint::ComputeDistinctiveDescriptors: the rows it reads now
        if (g->bad[mp]) return;
        std::vector<int> rows;
        for (const Obs &o : obs[mp])
            for (int s = 0; s < 4; ++s)
                if (o.idx[s] != -1) rows.push_back((int)row_of(o.kf, o.idx[s]));
        if (rows.empty()) return;
        pending[mp] = std::move(rows);
        ++ver[mp];
    }
    void replace(int a, int b) {   // a->Replace(b) (MapPoint.cc:316-380)
        log(1, a, b, -1);
        if (a == b) return;
        std::vector<Obs> o = std::move(obs[a]);
        obs[a].clear();
        g->bad[a] = 1;
        g->replaced[a] = b;
        for (const Obs &e : o) {
            int *row = kfmp(e.kf);
            if (!in_kf(b, e.kf)) {
                for (int s = 0; s < 4; ++s)
                    if (e.idx[s] != -1) row[e.idx[s]] = b, add_observation(b, e.kf, e.idx[s]);
            } else {
                for (int s = 0; s < 4; ++s)
                    if (e.idx[s] != -1) row[e.idx[s]] = -1;
            }
        }
        compute_distinctive(b);
    }

    omv_status scratch(size_t n_i32) {
        if (d_cap >= n_i32) return OMV_OK;
        if (d_i32) HIP_OK(hipFreeAsync(d_i32, st));
        d_i32 = nullptr;
        d_cap = std::max(n_i32, 2 * d_cap);
        HIP_OK(hipMallocAsync((void **)&d_i32, sizeof(int32_t) * d_cap, st));
        return OMV_OK;
    }
    // the pending descriptor recomputations, on the device, into the map-point table
    omv_status flush() {
        if (pending.empty()) return OMV_OK;
        std::vector<int32_t> h;   // [n mp | n + 1 start | rows | n best]
        const int n = (int)pending.size();
        std::vector<int32_t> start(1, 0), rows, mpl;
        for (auto &kv : pending) {
            mpl.push_back(kv.first);
            rows.insert(rows.end(), kv.second.begin(), kv.second.end());
            start.push_back((int32_t)rows.size());
        }
        h.insert(h.end(), mpl.begin(), mpl.end());
        h.insert(h.end(), start.begin(), start.end());
        h.insert(h.end(), rows.begin(), rows.end());
        OMV_OK_OR_RETURN(scratch(h.size() + n));
        HIP_OK(hipMemcpyAsync(d_i32, h.data(), sizeof(int32_t) * h.size(), hipMemcpyHostToDevice, st));
        int32_t *d_mp = d_i32, *d_start = d_mp + n, *d_rows = d_start + n + 1, *d_best = d_rows + rows.size();
        OMV_OK_OR_RETURN(omv_mappoint_distinctive_descriptors(n, d_start, d_rows, desc, d_best, nullptr, st));
        fuse_desc_scatter_kernel<<<(n + 3) / 4, 32, 0, st>>>(n, d_mp, d_best, desc, const_cast<uint8_t *>(mps->desc));
        HIP_OK(hipGetLastError());
        pending.clear();
        return OMV_OK;
    }
    // the window searches of `sel` (entries of `E`) with the current descriptors
    omv_status evaluate(std::vector<Entry> &E, const std::vector<int> &sel, const std::vector<std::pair<int, int>> &jobs) {
        if (sel.empty()) return OMV_OK;
        OMV_OK_OR_RETURN(flush());
        const size_t cap = std::max<size_t>(1, omv::matcher_kf_entry_cap(m));
        for (size_t s0 = 0; s0 < sel.size(); s0 += cap) {
            const size_t n = std::min(cap, sel.size() - s0);
            std::vector<omv_kf_search_job> js;
            std::vector<int32_t> list(n);
            for (size_t k = 0; k < n; ++k) {
                const Entry &e = E[sel[s0 + k]];
                list[k] = e.mp;
                if (js.empty() || js.back().kf != jobs[e.job].first || js.back().cam != jobs[e.job].second ||
                    (k > 0 && E[sel[s0 + k - 1]].job != e.job)) {
                    omv_kf_search_job J{};
                    J.kf = jobs[e.job].first, J.cam = jobs[e.job].second;
                    J.Tcw = g->Tcw[(size_t)J.kf * C + J.cam];
                    for (int q = 0; q < 3; ++q) J.Ow[q] = g->Ow[((size_t)J.kf * C + J.cam) * 3 + q];
                    J.mp_start = (int)k, J.mp_count = 0;
                    js.push_back(J);
                }
                ++js.back().mp_count;
            }
            OMV_OK_OR_RETURN(scratch(3 * n + js.size()));
            int32_t *d_list = d_i32, *d_bi = d_list + n, *d_bd = d_bi + n, *d_nm = d_bd + n;
            HIP_OK(hipMemcpyAsync(d_list, list.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, st));
            OMV_OK_OR_RETURN(omv_matcher_search_kf(m, n_kf, geom, kps, desc, n_kp_dev, (int)js.size(), js.data(), (int)n,
                                                   d_list, mps, &p, nullptr, d_bi, d_bd, d_nm, st));
            std::vector<int32_t> out(2 * n);
            HIP_OK(hipMemcpyAsync(out.data(), d_bi, sizeof(int32_t) * 2 * n, hipMemcpyDeviceToHost, st));
            HIP_OK(hipStreamSynchronize(st));
            ++n_calls;
            for (size_t k = 0; k < n; ++k) {
                Entry &e = E[sel[s0 + k]];
                e.best_idx = out[k], e.best_dist = out[n + k], e.ver = ver[e.mp];
            }
        }
        return OMV_OK;
    }
    // One phase: Fuse(kf, list, 3, cam) for each (kf, cam) of `jobs` in order, every call over the same `list`.
    omv_status phase(const std::vector<std::pair<int, int>> &jobs, const std::vector<int> &list, int32_t *n_fused) {
        // entries: the points a call can act on; a point bad or already in the keyframe now stays skipped
        std::vector<Entry> E;
        std::vector<int> job_lo(jobs.size() + 1, 0);
        for (size_t j = 0; j < jobs.size(); ++j) {
            job_lo[j] = (int)E.size();
            for (int mp : list)
                if (mp >= 0 && !g->bad[mp] && !in_kf(mp, jobs[j].first)) E.push_back(Entry{(int)j, mp, -1, -1, -1});
        }
        job_lo[jobs.size()] = (int)E.size();
        std::vector<int> sel(E.size());
        for (size_t k = 0; k < E.size(); ++k) sel[k] = (int)k;
        OMV_OK_OR_RETURN(evaluate(E, sel, jobs));
        for (size_t j = 0; j < jobs.size(); ++j) {
            const int kf = jobs[j].first;
            // stale entries of the rest of the phase, together
            sel.clear();
            for (int k = job_lo[j]; k < (int)E.size(); ++k)
                if (E[k].ver != ver[E[k].mp] && !g->bad[E[k].mp]) sel.push_back(k);
            n_re += (int)sel.size();
            OMV_OK_OR_RETURN(evaluate(E, sel, jobs));
            int nf = 0;
            int *row = kfmp(kf);
            for (int k = job_lo[j]; k < job_lo[j + 1]; ++k) {
                Entry &e = E[k];
                const int mp = e.mp;
                if (g->bad[mp] || in_kf(mp, kf)) continue;   // (:1517-1523)
                if (e.ver != ver[mp]) {   // went stale inside this call: re-evaluate the call's rest that is stale
                    sel.clear();
                    for (int q = k; q < job_lo[j + 1]; ++q)
                        if (E[q].ver != ver[E[q].mp] && !g->bad[E[q].mp]) sel.push_back(q);
                    n_re += (int)sel.size();
                    OMV_OK_OR_RETURN(evaluate(E, sel, jobs));
                }
                if (e.best_idx < 0 || e.best_dist > kThLow) continue;   // (:1628)
                const int in = row[e.best_idx];
                if (in >= 0) {   // (:1629-1636)
                    if (!g->bad[in]) {
                        if (g->n_obs[in] > g->n_obs[mp]) replace(mp, in);
                        else replace(in, mp);
                    }
                } else {   // (:1638-1639)
                    log(0, mp, kf, e.best_idx);
                    add_observation(mp, kf, e.best_idx);
                    row[e.best_idx] = mp;
                }
                ++nf;
            }
            n_fused[j] = nf;
        }
        return OMV_OK;
    }
};

}  // namespace

extern "C" omv_status omv_search_in_neighbors_fuse(omv_matcher *m, const omv_frame_geom *geom, const omv_kp *kps,
                                                   const uint8_t *desc, const int *n_kp, int kp_cap, omv_fuse_graph *g,
                                                   int current, int n_targets, const int32_t *targets,
                                                   const omv_kf_mps *mps, const omv_kf_search_params *p,
                                                   int32_t *n_fused, void *stream) {
    if (!m || !geom || !kps || !desc || !n_kp || kp_cap <= 0 || !g || !mps || !p || !n_fused || n_targets < 0 ||
        (n_targets > 0 && !targets) || p->mode != OMV_KF_FUSE)
        return OMV_ERR_ARG;
    const int C = geom->n_cams;
    if (C < 1 || C > 4 || g->n_kf <= 0 || current < 0 || current >= g->n_kf || g->n_mps < 0 || !g->n_blocks ||
        !g->Tcw || !g->Ow || !g->kf_mps || (g->n_mps > 0 && (!g->bad || !g->n_obs || !g->replaced || !g->obs_start ||
                                                            !g->out_obs_start)))
        return OMV_ERR_ARG;
    for (int t = 0; t < n_targets; ++t)
        if (targets[t] < 0 || targets[t] >= g->n_kf) return OMV_ERR_ARG;
    for (int k = 0; k < g->n_kf; ++k)
        if (g->n_blocks[k] != 1 && g->n_blocks[k] != 2 && g->n_blocks[k] != 4) return OMV_ERR_ARG;
    Walk w;
    w.m = m, w.geom = geom, w.kps = kps, w.desc = desc, w.n_kp_dev = n_kp, w.kp_cap = kp_cap, w.C = C, w.n_kf = g->n_kf;
    w.g = g, w.mps = mps, w.p = *p, w.st = (hipStream_t)stream;
    w.nkp.resize((size_t)g->n_kf * C);
    HIP_OK(hipMemcpyAsync(w.nkp.data(), n_kp, sizeof(int) * w.nkp.size(), hipMemcpyDeviceToHost, w.st));
    HIP_OK(hipStreamSynchronize(w.st));
    w.obs.resize(g->n_mps);
    w.ver.assign(g->n_mps, 0);
    for (int mp = 0; mp < g->n_mps; ++mp) {
        g->replaced[mp] = -1;
        for (int r = g->obs_start[mp]; r < g->obs_start[mp + 1]; ++r) {
            Obs o{g->obs_kf[r], {g->obs_idx[4 * r], g->obs_idx[4 * r + 1], g->obs_idx[4 * r + 2], g->obs_idx[4 * r + 3]}};
            if (o.kf < 0 || o.kf >= g->n_kf) return OMV_ERR_ARG;
            w.obs[mp].push_back(o);
        }
        std::sort(w.obs[mp].begin(), w.obs[mp].end(), [](const Obs &a, const Obs &b) { return a.kf < b.kf; });
    }
    for (int t = 0; t < n_targets * C + C; ++t) n_fused[t] = 0;
    auto blocks = [&](int kf) { return g->n_blocks[kf]; };
    // phase A: the current keyframe's GetMapPointMatches() snapshot into every target, block by block (:839-853)
    {
        const int *row = w.kfmp(current);
        std::vector<int> list(row, row + w.n_of(current));
        // every target's calls form one phase: the list is the same snapshot for all of them
        std::vector<std::pair<int, int>> jobs;
        std::vector<int> slot;
        for (int t = 0; t < n_targets; ++t)
            for (int c = 0; c < blocks(targets[t]); ++c) jobs.push_back({targets[t], c}), slot.push_back(t * C + c);
        std::vector<int32_t> nf(jobs.size(), 0);
        OMV_OK_OR_RETURN(w.phase(jobs, list, nf.data()));
        for (size_t j = 0; j < jobs.size(); ++j) n_fused[slot[j]] = nf[j];
    }
    // phase B: the targets' points (after phase A: non-bad, first occurrence) into the current keyframe (:859-889)
    {
        std::vector<int> list;
        std::vector<char> seen(g->n_mps, 0);
        for (int t = 0; t < n_targets; ++t) {
            const int kf = targets[t];
            const int *row = w.kfmp(kf);
            for (int i = 0, n = w.n_of(kf); i < n; ++i) {
                const int mp = row[i];
                if (mp < 0 || g->bad[mp] || seen[mp]) continue;
                seen[mp] = 1;
                list.push_back(mp);
            }
        }
        std::vector<std::pair<int, int>> jobs;
        for (int c = 0; c < blocks(current); ++c) jobs.push_back({current, c});
        std::vector<int32_t> nf(jobs.size(), 0);
        OMV_OK_OR_RETURN(w.phase(jobs, list, nf.data()));
        for (size_t j = 0; j < jobs.size(); ++j) n_fused[n_targets * C + (int)j] = nf[j];
    }
    OMV_OK_OR_RETURN(w.flush());   // the last survivors' descriptors
    if (w.d_i32) HIP_OK(hipFreeAsync(w.d_i32, w.st));
    HIP_OK(hipStreamSynchronize(w.st));
    // final observations
    int rows = 0;
    for (int mp = 0; mp < g->n_mps; ++mp) {
        g->out_obs_start[mp] = rows;
        for (const Obs &o : w.obs[mp]) {
            if (rows < g->obs_cap && g->out_obs_kf && g->out_obs_idx) {
                g->out_obs_kf[rows] = o.kf;
                for (int s = 0; s < 4; ++s) g->out_obs_idx[4 * (size_t)rows + s] = o.idx[s];
            } else {
                w.overflow = true;
            }
            ++rows;
        }
    }
    if (g->n_mps >= 0) g->out_obs_start[g->n_mps] = rows;
    g->n_log = w.n_log, g->n_reevaluated = w.n_re, g->n_device_calls = w.n_calls;
    return w.overflow ? OMV_ERR_CAPACITY : OMV_OK;
}
