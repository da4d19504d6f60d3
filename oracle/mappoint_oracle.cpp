// TEST INFRASTRUCTURE ONLY — CPU restatement of MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:405-490)
// and MapPoint::UpdateNormalAndDepth (src/MapPoint.cc:503-588), written literally after the reference: the N x N
// float distance matrix, std::sort of each row, vDists[0.5 * (N - 1)], the first strict minimum; the normal and the
// distances in float with Eigen's 3-element expressions evaluated left to right.  Checker of
// openmavis_amd/csrc/mappoint.hip; never linked into the product.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <vector>

namespace {
int descriptor_distance(const uint8_t *a, const uint8_t *b) {   // ORBmatcher::DescriptorDistance (ORBmatcher.cc:2577-2591)
    const int32_t *pa = reinterpret_cast<const int32_t *>(a), *pb = reinterpret_cast<const int32_t *>(b);
    int dist = 0;
    for (int i = 0; i < 8; i++, pa++, pb++) {
        unsigned int v = *pa ^ *pb;
        v = v - ((v >> 1) & 0x55555555);
        v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
        dist += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
    }
    return dist;
}
}  // namespace

extern "C" {

void oracle_distinctive_descriptors(int n_points, const int32_t *desc_start, const int32_t *desc_row,
                                    const uint8_t *desc, int32_t *best_row) {
    for (int p = 0; p < n_points; ++p) {
        std::vector<const uint8_t *> vDescriptors;
        for (int e = desc_start[p]; e < desc_start[p + 1]; ++e) vDescriptors.push_back(desc + (size_t)desc_row[e] * 32);
        if (vDescriptors.empty()) {
            best_row[p] = -1;
            continue;
        }
        const size_t N = vDescriptors.size();
        std::vector<float> Distances(N * N);
        for (size_t i = 0; i < N; i++) {
            Distances[i * N + i] = 0;
            for (size_t j = i + 1; j < N; j++) {
                int distij = descriptor_distance(vDescriptors[i], vDescriptors[j]);
                Distances[i * N + j] = distij;
                Distances[j * N + i] = distij;
            }
        }
        int BestMedian = INT_MAX;
        int BestIdx = 0;
        for (size_t i = 0; i < N; i++) {
            std::vector<int> vDists(Distances.begin() + i * N, Distances.begin() + (i + 1) * N);
            std::sort(vDists.begin(), vDists.end());
            int median = vDists[0.5 * (N - 1)];
            if (median < BestMedian) {
                BestMedian = median;
                BestIdx = (int)i;
            }
        }
        best_row[p] = desc_row[desc_start[p] + BestIdx];
    }
}

void oracle_normal_depth(int n_points, const int32_t *obs_start, const float *obs_center, const float *pos,
                         const float *ref_center, const float *ref_level_scale, const float *ref_max_scale,
                         float *normal_out, float *min_dist, float *max_dist) {
    auto norm = [](float x, float y, float z) { return std::sqrt(x * x + y * y + z * z); };
    for (int p = 0; p < n_points; ++p) {
        if (obs_start[p + 1] == obs_start[p]) continue;
        const float *P = pos + 3 * p;
        float normal[3] = {0.f, 0.f, 0.f};
        int n = 0;
        for (int e = obs_start[p]; e < obs_start[p + 1]; ++e) {
            const float ni[3] = {P[0] - obs_center[3 * e], P[1] - obs_center[3 * e + 1], P[2] - obs_center[3 * e + 2]};
            const float r = norm(ni[0], ni[1], ni[2]);
            for (int q = 0; q < 3; ++q) normal[q] = normal[q] + ni[q] / r;
            n++;
        }
        const float PC[3] = {P[0] - ref_center[3 * p], P[1] - ref_center[3 * p + 1], P[2] - ref_center[3 * p + 2]};
        const float dist = norm(PC[0], PC[1], PC[2]);
        max_dist[p] = dist * ref_level_scale[p];
        min_dist[p] = max_dist[p] / ref_max_scale[p];
        for (int q = 0; q < 3; ++q) normal_out[3 * p + q] = normal[q] / n;
    }
}

}  // extern "C"
