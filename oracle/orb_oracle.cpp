// =====================================================================================================
// TEST INFRASTRUCTURE ONLY — CPU oracle for the ORB front-end. Never linked into the product path.
//
// A from-scratch, scalar C++ restatement of the reference extractor
//   /root/reference/src/ORBextractor.cc  (ORBextractor ctor :351-414, IC_Angle :19-43,
//   computeOrbDescriptor :46-90, DivideNode :425-480, compareNodes :482-494,
//   DistributeOctTree :496-702, ComputeKeyPointsOctTree :704-823, operator() :987-1071,
//   ComputePyramid :1073-1104)
// together with the OpenCV 4.x primitives it calls, restated from their published algorithms
// (OpenCV is not vendored in the reference and is absent here):
//   cv::resize INTER_LINEAR (8U fixed-point path, 11-bit coefficients),
//   cv::FAST TYPE_9_16 + cornerScore<16> + 3x3 NMS,
//   cv::GaussianBlur 7x7 sigma 2 (8U bit-exact path, error-diffused 8-bit kernel),
//   cv::fastAtan2, cvRound (round-half-even).
// The octree is restated with std::list / std::sort exactly as the reference uses them, so the
// libstdc++ introsort tie order is reproduced by the library itself (the GPU path has its own
// replica and is checked against this).  sin/cos are the host libm cosf/sinf, as in the
// reference (computeOrbDescriptor :49).
//
// Parity status: the reference cannot be built here (OpenCV/Eigen/Pangolin absent);
// no reference test holds fixtures for this path.  Parity against real OpenCV is therefore
// UNPINNED; this oracle pins the restated semantics documented in DESIGN.md.
// Build: oracle/Makefile  (g++ -O2 -ffp-contract=off, no fast-math).
// =====================================================================================================
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <list>
#include <thread>
#include <vector>

namespace oracle {

static const int kPatch = 31, kHalfPatch = 15, kEdge = 19;

static const int kPattern[256 * 4] = {
#define OMV_PATTERN_TABLE_BEGIN
#define OMV_PATTERN_TABLE_END
#include "../openmavis_amd/csrc/orb_pattern_31.inc"
};

// ---- OpenCV scalar helpers ----------------------------------------------------------------------
static inline int round_even(float v) { return (int)std::nearbyint(v); }   // cvRound (SSE2 cvtss2si)
static inline int round_even_d(double v) { return (int)std::nearbyint(v); }

// cv::fastAtan2 — OpenCV 4.x atan_f32 (degrees), computed in float, no contraction.
static float fast_atan2_deg(float y, float x) {
    const float k1 = 0.9997878412794807f * (float)(180 / M_PI);
    const float k3 = -0.3258083974640975f * (float)(180 / M_PI);
    const float k5 = 0.1555786518463281f * (float)(180 / M_PI);
    const float k7 = -0.04432655554792128f * (float)(180 / M_PI);
    float ax = std::fabs(x), ay = std::fabs(y), a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((k7 * c2 + k5) * c2 + k3) * c2 + k1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((k7 * c2 + k5) * c2 + k3) * c2 + k1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

struct KP {
    float x, y, size, angle, response;
    int octave;
};

struct Img {   // owning u8 image
    int w = 0, h = 0;
    std::vector<uint8_t> px;
    uint8_t at(int y, int x) const { return px[(size_t)y * w + x]; }
};

// ---- cv::resize INTER_LINEAR, 8U fixed point ------------------------------------------------------
static void resize_linear_u8(const Img &src, Img &dst, int dw, int dh) {
    dst.w = dw;
    dst.h = dh;
    dst.px.assign((size_t)dw * dh, 0);
    const int sw = src.w, sh = src.h;
    const double sx_scale = 1.0 / ((double)dw / sw), sy_scale = 1.0 / ((double)dh / sh);
    std::vector<int> xo(dw), yo(dh);
    std::vector<short> xa(2 * dw), yb(2 * dh);
    int xmax = dw;
    for (int dx = 0; dx < dw; ++dx) {
        float fx = (float)((dx + 0.5) * sx_scale - 0.5);
        int sx = (int)std::floor(fx);
        fx -= sx;
        if (sx < 0) fx = 0, sx = 0;
        if (sx + 1 >= sw) {
            xmax = std::min(xmax, dx);
            if (sx >= sw - 1) fx = 0, sx = sw - 1;
        }
        xo[dx] = sx;
        xa[2 * dx] = (short)round_even((1.f - fx) * 2048.f);
        xa[2 * dx + 1] = (short)round_even(fx * 2048.f);
    }
    for (int dy = 0; dy < dh; ++dy) {
        float fy = (float)((dy + 0.5) * sy_scale - 0.5);
        int sy = (int)std::floor(fy);
        fy -= sy;
        yo[dy] = sy;
        yb[2 * dy] = (short)round_even((1.f - fy) * 2048.f);
        yb[2 * dy + 1] = (short)round_even(fy * 2048.f);
    }
    std::vector<int> r0(dw), r1(dw);
    auto hrow = [&](int sy, std::vector<int> &out) {
        sy = std::min(std::max(sy, 0), sh - 1);
        const uint8_t *S = &src.px[(size_t)sy * sw];
        for (int dx = 0; dx < dw; ++dx) {
            int sx = xo[dx];
            out[dx] = dx < xmax ? S[sx] * xa[2 * dx] + S[sx + 1] * xa[2 * dx + 1] : S[sx] * 2048;
        }
    };
    for (int dy = 0; dy < dh; ++dy) {
        hrow(yo[dy], r0);
        hrow(yo[dy] + 1, r1);
        int b0 = yb[2 * dy], b1 = yb[2 * dy + 1];
        uint8_t *D = &dst.px[(size_t)dy * dw];
        for (int dx = 0; dx < dw; ++dx) {
            int v = (((b0 * (r0[dx] >> 4)) >> 16) + ((b1 * (r1[dx] >> 4)) >> 16) + 2) >> 2;
            D[dx] = (uint8_t)std::min(v, 255);
        }
    }
}

// ---- cv::FAST TYPE_9_16 with NMS on a sub-image [y0,y1) x [x0,x1) --------------------------------
static const int kRing[16][2] = {{0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1}, {2, -2}, {1, -3},
                                 {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

static int corner_score16(const Img &im, int y, int x, int threshold) {
    int v = im.at(y, x);
    int d[25];
    for (int k = 0; k < 25; ++k) d[k] = v - im.at(y + kRing[k & 15][1], x + kRing[k & 15][0]);
    int a0 = threshold;
    for (int k = 0; k < 16; k += 2) {
        int a = std::min(d[k + 1], std::min(d[k + 2], d[k + 3]));
        if (a <= a0) continue;
        for (int m = 4; m <= 8; ++m) a = std::min(a, d[k + m]);
        a0 = std::max(a0, std::min(a, d[k]));
        a0 = std::max(a0, std::min(a, d[k + 9]));
    }
    int b0 = -a0;
    for (int k = 0; k < 16; k += 2) {
        int b = d[k + 1];
        for (int m = 2; m <= 5; ++m) b = std::max(b, d[k + m]);
        if (b >= b0) continue;
        for (int m = 6; m <= 8; ++m) b = std::max(b, d[k + m]);
        b0 = std::min(b0, std::max(b, d[k]));
        b0 = std::min(b0, std::max(b, d[k + 9]));
    }
    return -b0 - 1;
}

// Keypoints in sub-image coordinates, emitted row-major like FAST_t<16>.
static void fast9(const Img &im, int y0, int y1, int x0, int x1, int threshold, std::vector<KP> &out) {
    out.clear();
    const int rows = y1 - y0, cols = x1 - x0;
    threshold = std::min(std::max(threshold, 0), 255);
    if (rows < 7 || cols < 7) return;
    std::vector<int> score((size_t)rows * cols, 0);
    std::vector<char> is_corner((size_t)rows * cols, 0);
    for (int i = 3; i < rows - 3; ++i)
        for (int j = 3; j < cols - 3; ++j) {
            int v = im.at(y0 + i, x0 + j);
            int nd = 0, nb = 0, best_d = 0, best_b = 0;
            for (int k = 0; k < 25; ++k) {
                int p = im.at(y0 + i + kRing[k & 15][1], x0 + j + kRing[k & 15][0]);
                nd = p < v - threshold ? nd + 1 : 0;
                nb = p > v + threshold ? nb + 1 : 0;
                best_d = std::max(best_d, nd);
                best_b = std::max(best_b, nb);
            }
            if (best_d > 8 || best_b > 8) {
                is_corner[(size_t)i * cols + j] = 1;
                score[(size_t)i * cols + j] = corner_score16(im, y0 + i, x0 + j, threshold);
            }
        }
    for (int i = 3; i < rows - 3; ++i)
        for (int j = 3; j < cols - 3; ++j) {
            if (!is_corner[(size_t)i * cols + j]) continue;
            int s = score[(size_t)i * cols + j];
            bool keep = true;
            for (int dy = -1; dy <= 1 && keep; ++dy)
                for (int dx = -1; dx <= 1; ++dx)
                    if ((dy || dx) && !(s > score[(size_t)(i + dy) * cols + j + dx])) { keep = false; break; }
            if (keep) out.push_back(KP{(float)j, (float)i, 7.f, -1.f, (float)s, 0});
        }
}

// ---- quad-tree distribution (ORBextractor.cc:425-702), restated with std::list/std::sort ----------
struct QNode {
    std::vector<KP> keys;
    int ulx, uly, urx, ury, blx, bly, brx, bry;
    std::list<QNode>::iterator self;
    bool leaf = false;
};

static void split4(const QNode &p, QNode &a, QNode &b, QNode &c, QNode &d) {
    const int hx = (int)std::ceil((float)(p.urx - p.ulx) / 2);
    const int hy = (int)std::ceil((float)(p.bry - p.uly) / 2);
    a.ulx = p.ulx, a.uly = p.uly, a.urx = p.ulx + hx, a.ury = p.uly;
    a.blx = p.ulx, a.bly = p.uly + hy, a.brx = p.ulx + hx, a.bry = p.uly + hy;
    b.ulx = a.urx, b.uly = a.ury, b.urx = p.urx, b.ury = p.ury;
    b.blx = a.brx, b.bly = a.bry, b.brx = p.urx, b.bry = p.uly + hy;
    c.ulx = a.blx, c.uly = a.bly, c.urx = a.brx, c.ury = a.bry;
    c.blx = p.blx, c.bly = p.bly, c.brx = a.brx, c.bry = p.bly;
    d.ulx = c.urx, d.uly = c.ury, d.urx = b.brx, d.ury = b.bry;
    d.blx = c.brx, d.bly = c.bry, d.brx = p.brx, d.bry = p.bry;
    for (const KP &k : p.keys) {
        if (k.x < a.urx) (k.y < a.bry ? a : c).keys.push_back(k);
        else (k.y < a.bry ? b : d).keys.push_back(k);
    }
    for (QNode *n : {&a, &b, &c, &d})
        if (n->keys.size() == 1) n->leaf = true;
}

static bool node_less(std::pair<int, QNode *> &l, std::pair<int, QNode *> &r) {
    if (l.first != r.first) return l.first < r.first;
    return l.second->ulx < r.second->ulx;
}

static std::vector<KP> distribute(const std::vector<KP> &pts, int minX, int maxX, int minY, int maxY,
                                  int N) {
    const int nIni = (int)std::round((float)(maxX - minX) / (maxY - minY));
    const float hX = (float)(maxX - minX) / nIni;
    std::list<QNode> nodes;
    std::vector<QNode *> ini(nIni);
    for (int i = 0; i < nIni; ++i) {
        QNode q;
        q.ulx = (int)(hX * (float)i), q.uly = 0;
        q.urx = (int)(hX * (float)(i + 1)), q.ury = 0;
        q.blx = q.ulx, q.bly = maxY - minY;
        q.brx = q.urx, q.bry = maxY - minY;
        nodes.push_back(q);
        ini[i] = &nodes.back();
    }
    for (const KP &k : pts) ini[(size_t)(k.x / hX)]->keys.push_back(k);
    for (auto it = nodes.begin(); it != nodes.end();) {
        if (it->keys.size() == 1) { it->leaf = true; ++it; }
        else if (it->keys.empty()) it = nodes.erase(it);
        else ++it;
    }
    bool done = false;
    std::vector<std::pair<int, QNode *>> expandable;
    // push the non-empty children of `p` to the front; the ones with >1 key become expandable
    auto emit_children = [&](QNode &p, std::vector<std::pair<int, QNode *>> &exp, int *nexp) {
        QNode kids[4];
        split4(p, kids[0], kids[1], kids[2], kids[3]);
        for (QNode &k : kids) {
            if (k.keys.empty()) continue;
            nodes.push_front(k);
            if (k.keys.size() > 1) {
                if (nexp) ++*nexp;
                exp.push_back({(int)k.keys.size(), &nodes.front()});
                nodes.front().self = nodes.begin();
            }
        }
    };
    while (!done) {
        int prev = (int)nodes.size();
        int nexp = 0;
        expandable.clear();
        for (auto it = nodes.begin(); it != nodes.end();) {
            if (it->leaf) { ++it; continue; }
            emit_children(*it, expandable, &nexp);
            it = nodes.erase(it);
        }
        if ((int)nodes.size() >= N || (int)nodes.size() == prev) {
            done = true;
        } else if ((int)nodes.size() + nexp * 3 > N) {
            while (!done) {
                prev = (int)nodes.size();
                std::vector<std::pair<int, QNode *>> cur = expandable;
                expandable.clear();
                std::sort(cur.begin(), cur.end(), node_less);
                for (int j = (int)cur.size() - 1; j >= 0; --j) {
                    emit_children(*cur[j].second, expandable, nullptr);
                    nodes.erase(cur[j].second->self);
                    if ((int)nodes.size() >= N) break;
                }
                if ((int)nodes.size() >= N || (int)nodes.size() == prev) done = true;
            }
        }
    }
    std::vector<KP> res;
    for (QNode &q : nodes) {
        const KP *best = &q.keys[0];
        for (size_t k = 1; k < q.keys.size(); ++k)
            if (q.keys[k].response > best->response) best = &q.keys[k];
        res.push_back(*best);
    }
    return res;
}

// ---- intensity-centroid angle (ORBextractor.cc:19-43) ----------------------------------------------
static float ic_angle(const Img &im, float px, float py, const int *umax) {
    int cy = round_even(py), cx = round_even(px);
    int m01 = 0, m10 = 0;
    for (int u = -kHalfPatch; u <= kHalfPatch; ++u) m10 += u * im.at(cy, cx + u);
    for (int v = 1; v <= kHalfPatch; ++v) {
        int vs = 0, d = umax[v];
        for (int u = -d; u <= d; ++u) {
            int p = im.at(cy + v, cx + u), m = im.at(cy - v, cx + u);
            vs += p - m;
            m10 += u * (p + m);
        }
        m01 += v * vs;
    }
    return fast_atan2_deg((float)m01, (float)m10);
}

// ---- cv::GaussianBlur 7x7 sigma=2, 8U bit-exact fixed point, BORDER_REFLECT_101 -------------------
static const int kGauss7[7] = {18, 34, 48, 56, 48, 34, 18};   // error-diffused 8-bit kernel
static inline int reflect101(int p, int n) {
    while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
    return p;
}
static void gauss7_u8(const Img &src, Img &dst) {
    const int w = src.w, h = src.h;
    std::vector<int> tmp((size_t)w * h);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            int s = 0;
            for (int k = 0; k < 7; ++k) s += kGauss7[k] * src.at(y, reflect101(x + k - 3, w));
            tmp[(size_t)y * w + x] = s;   // ufixedpoint16: 8 fractional bits, exact
        }
    dst.w = w, dst.h = h;
    dst.px.assign((size_t)w * h, 0);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            uint32_t s = 0;
            for (int k = 0; k < 7; ++k) s += (uint32_t)kGauss7[k] * tmp[(size_t)reflect101(y + k - 3, h) * w + x];
            dst.px[(size_t)y * w + x] = (uint8_t)std::min<uint32_t>((s + (1u << 15)) >> 16, 255u);
        }
}

// Floating-point contraction study (tools/fma_study.py): 0 = none (the parity mode: every restated float path
// rounds each operation, as the device does); 1 = the contraction GCC applies to the reference's own
// translation unit when built with its flags (-O3 -march=native on an FMA machine, CMakeLists.txt:12-15): the
// steering products of GET_VALUE (ORBextractor.cc:56-57) fused as GCC's convert_mult_to_fma does (the first
// product of `a*b + c*d` / `a*b - c*d` becomes the FMA, the second is rounded).  OpenCV's own code (fastAtan2,
// resize, FAST, GaussianBlur) keeps mode 0: its contraction depends on how OpenCV was built (unpinned).
static int g_contract = 0;
extern "C" void oracle_set_contract(int mode) { g_contract = mode; }

// ---- steered BRIEF (ORBextractor.cc:46-90) ---------------------------------------------------------
static void rbrief(const Img &blur, const KP &k, uint8_t *desc) {
    const float rad = k.angle * (float)(M_PI / 180.f);
    const float a = cosf(rad), b = sinf(rad);
    const int cy = round_even(k.y), cx = round_even(k.x);
    auto sample = [&](int idx) {
        const int px = kPattern[2 * idx], py = kPattern[2 * idx + 1];
        int dy, dx;
        if (g_contract == 1) {
            dy = round_even(std::fma((float)px, b, (float)py * a));
            dx = round_even(std::fma((float)px, a, -((float)py * b)));
        } else {
            dy = round_even((float)px * b + (float)py * a);
            dx = round_even((float)px * a - (float)py * b);
        }
        return (int)blur.at(cy + dy, cx + dx);
    };
    for (int byte = 0; byte < 32; ++byte) {
        int v = 0;
        for (int bit = 0; bit < 8; ++bit) {
            int s = byte * 16 + bit * 2;
            v |= (sample(s) < sample(s + 1)) << bit;
        }
        desc[byte] = (uint8_t)v;
    }
}

// ---- the extractor -----------------------------------------------------------------------------------
struct Extractor {
    int nfeatures, nlevels, iniTh, minTh;
    double scaleFactor;
    std::vector<float> scale, invScale, sigma2, invSigma2;
    std::vector<int> quota;
    int umax[kHalfPatch + 1];

    Extractor(int nf, float sf, int nl, int ini, int mn)
        : nfeatures(nf), nlevels(nl), iniTh(ini), minTh(mn), scaleFactor(sf) {
        scale.assign(nl, 1.f), sigma2.assign(nl, 1.f), invScale.resize(nl), invSigma2.resize(nl);
        for (int i = 1; i < nl; ++i) {
            scale[i] = (float)(scale[i - 1] * scaleFactor);   // float * double, as the reference
            sigma2[i] = scale[i] * scale[i];
        }
        for (int i = 0; i < nl; ++i) invScale[i] = 1.0f / scale[i], invSigma2[i] = 1.0f / sigma2[i];
        quota.assign(nl, 0);
        const float f = (float)(1.0f / scaleFactor);
        float per = nf * (1 - f) / (1 - (float)std::pow((double)f, (double)nl));
        int sum = 0;
        for (int l = 0; l < nl - 1; ++l) {
            quota[l] = round_even(per);
            sum += quota[l];
            per *= f;
        }
        quota[nl - 1] = std::max(nf - sum, 0);
        const int vmax = (int)std::floor(kHalfPatch * std::sqrt(2.f) / 2 + 1);
        const int vmin = (int)std::ceil(kHalfPatch * std::sqrt(2.f) / 2);
        for (int v = 0; v <= vmax; ++v) umax[v] = round_even_d(std::sqrt((double)kHalfPatch * kHalfPatch - v * v));
        for (int v = kHalfPatch, v0 = 0; v >= vmin; --v) {
            while (umax[v0] == umax[v0 + 1]) ++v0;
            umax[v] = v0;
            ++v0;
        }
    }

    void level_size(int W, int H, int l, int &w, int &h) const {
        w = round_even((float)W * invScale[l]);
        h = round_even((float)H * invScale[l]);
    }

    void pyramid(const Img &im, std::vector<Img> &pyr) const {
        pyr.assign(nlevels, Img());
        pyr[0] = im;
        for (int l = 1; l < nlevels; ++l) {
            int w, h;
            level_size(im.w, im.h, l, w, h);
            if (w == pyr[l - 1].w && h == pyr[l - 1].h) pyr[l] = pyr[l - 1];
            else resize_linear_u8(pyr[l - 1], pyr[l], w, h);
        }
    }

    // Candidate keypoints of one level, in vToDistributeKeys order (ORBextractor.cc:709-794).
    void level_candidates(const Img &L, std::vector<KP> &cand) const {
        cand.clear();
        const float W = 35;
        const int minB = kEdge - 3, maxBX = L.w - kEdge + 3, maxBY = L.h - kEdge + 3;
        const float width = (float)(maxBX - minB), height = (float)(maxBY - minB);
        const int nCols = (int)(width / W), nRows = (int)(height / W);
        const int wCell = (int)std::ceil(width / nCols), hCell = (int)std::ceil(height / nRows);
        std::vector<KP> cell;
        for (int i = 0; i < nRows; ++i) {
            const float iniY = (float)(minB + i * hCell);
            float maxY = iniY + hCell + 6;
            if (iniY >= maxBY - 3) continue;
            if (maxY > maxBY) maxY = (float)maxBY;
            for (int j = 0; j < nCols; ++j) {
                const float iniX = (float)(minB + j * wCell);
                float maxX = iniX + wCell + 6;
                if (iniX >= maxBX - 6) continue;
                if (maxX > maxBX) maxX = (float)maxBX;
                fast9(L, (int)iniY, (int)maxY, (int)iniX, (int)maxX, iniTh, cell);
                if (cell.empty()) fast9(L, (int)iniY, (int)maxY, (int)iniX, (int)maxX, minTh, cell);
                for (KP k : cell) {
                    k.x += j * wCell;
                    k.y += i * hCell;
                    cand.push_back(k);
                }
            }
        }
    }

    // Distributed keypoints of one level (level coordinates, angle set).
    void level_keypoints(const Img &L, int level, std::vector<KP> &kps) const {
        std::vector<KP> cand;
        level_candidates(L, cand);
        const int minB = kEdge - 3, maxBX = L.w - kEdge + 3, maxBY = L.h - kEdge + 3;
        kps = distribute(cand, minB, maxBX, minB, maxBY, quota[level]);
        const int psz = (int)(kPatch * scale[level]);
        for (KP &k : kps) {
            k.x += minB;
            k.y += minB;
            k.octave = level;
            k.size = (float)psz;
        }
        for (KP &k : kps) k.angle = ic_angle(L, k.x, k.y, umax);
    }

    // ORBextractor::operator() — returns monoIndex; kps/desc sized to the keypoint count.
    int extract(const Img &im, int lap0, int lap1, std::vector<KP> &out, std::vector<uint8_t> &desc) const {
        std::vector<Img> pyr;
        pyramid(im, pyr);
        std::vector<std::vector<KP>> all(nlevels);
        for (int l = 0; l < nlevels; ++l) level_keypoints(pyr[l], l, all[l]);
        int total = 0;
        for (auto &v : all) total += (int)v.size();
        out.assign(total, KP{});
        desc.assign((size_t)total * 32, 0);
        int mono = 0, stereo = total - 1;
        for (int l = 0; l < nlevels; ++l) {
            if (all[l].empty()) continue;
            Img blur;
            gauss7_u8(pyr[l], blur);
            const float s = scale[l];
            for (KP k : all[l]) {
                uint8_t d[32];
                rbrief(blur, k, d);
                if (l != 0) k.x *= s, k.y *= s;
                int slot = (k.x >= lap0 && k.x <= lap1) ? stereo-- : mono++;
                out[slot] = k;
                std::memcpy(&desc[(size_t)slot * 32], d, 32);
            }
        }
        return mono;
    }
};

}  // namespace oracle

// ===================================== C ABI for ctypes ===========================================
extern "C" {

struct oracle_kp {
    float x, y, size, angle, response;
    int32_t octave;
};

// libstdc++'s std::sort itself with compareNodes' order (src/ORBextractor.cc:482-494: size, then UL.x;
// ties left to the algorithm): the expected permutation for omv_selftest_node_sort.
int oracle_std_sort_pairs(const int *k1, const int *k2, int n, int *perm) {
    struct E { int a, b, id; };
    std::vector<E> v(n);
    for (int i = 0; i < n; ++i) v[i] = E{k1[i], k2[i], i};
    std::sort(v.begin(), v.end(), [](const E &x, const E &y) { return x.a < y.a || (x.a == y.a && x.b < y.b); });
    for (int i = 0; i < n; ++i) perm[i] = v[i].id;
    return 0;
}

static oracle::Img wrap(const uint8_t *img, int w, int h, int stride) {
    oracle::Img im;
    im.w = w, im.h = h;
    im.px.resize((size_t)w * h);
    for (int y = 0; y < h; ++y) std::memcpy(&im.px[(size_t)y * w], img + (size_t)y * stride, w);
    return im;
}

// Scale tables / quotas / umax (ctor KATs).
void oracle_orb_tables(int nf, float sf, int nl, float *scale, float *inv_scale, float *sigma2,
                       float *inv_sigma2, int *quota, int *umax) {
    oracle::Extractor ex(nf, sf, nl, 20, 7);
    for (int l = 0; l < nl; ++l) {
        scale[l] = ex.scale[l], inv_scale[l] = ex.invScale[l], sigma2[l] = ex.sigma2[l];
        inv_sigma2[l] = ex.invSigma2[l], quota[l] = ex.quota[l];
    }
    for (int v = 0; v <= oracle::kHalfPatch; ++v) umax[v] = ex.umax[v];
}

// Pyramid level l of an image into out (w_l*h_l bytes).  Returns 0.
int oracle_orb_pyramid_level(const uint8_t *img, int w, int h, int stride, int nf, float sf, int nl,
                             int level, uint8_t *out, int *ow, int *oh) {
    oracle::Extractor ex(nf, sf, nl, 20, 7);
    std::vector<oracle::Img> pyr;
    ex.pyramid(wrap(img, w, h, stride), pyr);
    *ow = pyr[level].w, *oh = pyr[level].h;
    if (out) std::memcpy(out, pyr[level].px.data(), pyr[level].px.size());
    return 0;
}

// Harris response at integer level positions (x, y): OpenCV ORB's HarrisResponses (modules/features2d/src/orb.cpp,
// blockSize 7, harris_k 0.04) restated -- the north star's "Harris score"; the reference itself never computes it
// (HARRIS_SCORE is a dead enum, include/ORBextractor.h:24; its response is FAST's).  Sobel-like Ix / Iy over the 7x7
// block, integer sums a, b, c, then ((float)a * b - (float)c * c - k ((float)a + b)^2) * scale^4 in float.
// Parity unpinned (no OpenCV build here): the restatement is checked against an independent numpy form in tests.
void oracle_harris_responses(const uint8_t *lvl, int w, int h, int stride, const int *xs, const int *ys, int n,
                             float *out) {
    (void)w, (void)h;
    const int bs = 7, r = bs / 2;
    const float scale = 1.f / ((1 << 2) * bs * 255.f);
    const float scale_sq_sq = scale * scale * scale * scale;
    const float harris_k = 0.04f;
    for (int q = 0; q < n; ++q) {
        int a = 0, b = 0, c = 0;
        for (int i = 0; i < bs; ++i)
            for (int j = 0; j < bs; ++j) {
                const uint8_t *p = lvl + (size_t)(ys[q] - r + i) * stride + (xs[q] - r + j);
                const int Ix = (p[1] - p[-1]) * 2 + (p[-stride + 1] - p[-stride - 1]) + (p[stride + 1] - p[stride - 1]);
                const int Iy = (p[stride] - p[-stride]) * 2 + (p[stride - 1] - p[-stride - 1]) + (p[stride + 1] - p[-stride + 1]);
                a += Ix * Ix;
                b += Iy * Iy;
                c += Ix * Iy;
            }
        out[q] = ((float)a * b - (float)c * c - harris_k * ((float)a + b) * ((float)a + b)) * scale_sq_sq;
    }
}

// FAST candidates (vToDistributeKeys order) of one level given the level image. Returns count.
int oracle_orb_level_candidates(const uint8_t *lvl, int w, int h, int iniTh, int minTh, float *xs,
                                float *ys, float *resp, int cap) {
    oracle::Extractor ex(1000, 1.2f, 8, iniTh, minTh);
    oracle::Img L = wrap(lvl, w, h, w);
    std::vector<oracle::KP> cand;
    ex.level_candidates(L, cand);
    int n = (int)cand.size();
    for (int i = 0; i < n && i < cap; ++i) xs[i] = cand[i].x, ys[i] = cand[i].y, resp[i] = cand[i].response;
    return n;
}

// Octree distribution of a candidate list; returns the selected candidate indices in output order.
int oracle_orb_distribute(const float *xs, const float *ys, const float *resp, int n, int minX, int maxX,
                          int minY, int maxY, int N, int *sel, int cap) {
    std::vector<oracle::KP> pts(n);
    for (int i = 0; i < n; ++i) pts[i] = oracle::KP{xs[i], ys[i], 7.f, -1.f, resp[i], i};   // octave = id
    std::vector<oracle::KP> r = oracle::distribute(pts, minX, maxX, minY, maxY, N);
    for (size_t i = 0; i < r.size() && (int)i < cap; ++i) sel[i] = r[i].octave;
    return (int)r.size();
}

// Full ORBextractor::operator() on one image. Returns the keypoint count; *mono = monoIndex.
int oracle_orb_extract(const uint8_t *img, int w, int h, int stride, int nf, float sf, int nl, int iniTh,
                       int minTh, int lap0, int lap1, oracle_kp *kps, uint8_t *desc, int cap, int *mono) {
    oracle::Extractor ex(nf, sf, nl, iniTh, minTh);
    std::vector<oracle::KP> out;
    std::vector<uint8_t> d;
    *mono = ex.extract(wrap(img, w, h, stride), lap0, lap1, out, d);
    int n = (int)out.size();
    for (int i = 0; i < n && i < cap; ++i) {
        kps[i] = oracle_kp{out[i].x, out[i].y, out[i].size, out[i].angle, out[i].response, out[i].octave};
        std::memcpy(desc + (size_t)i * 32, &d[(size_t)i * 32], 32);
    }
    return n;
}

// Multi-camera frame, reference-faithful threading: one std::thread per camera (Frame.cc:1841-1862).
// imgs: n_cams pointers; outputs [cam][cap]. Returns 0.
int oracle_orb_extract_frame(int n_cams, const uint8_t *const *imgs, int w, int h, int stride, int nf,
                             float sf, int nl, int iniTh, int minTh, const int *lapping, oracle_kp *kps,
                             uint8_t *desc, int cap, int *n_out, int *mono, int threaded) {
    auto one = [&](int c) {
        n_out[c] = oracle_orb_extract(imgs[c], w, h, stride, nf, sf, nl, iniTh, minTh, lapping[2 * c],
                                      lapping[2 * c + 1], kps + (size_t)c * cap, desc + (size_t)c * cap * 32,
                                      cap, &mono[c]);
    };
    if (!threaded) {
        for (int c = 0; c < n_cams; ++c) one(c);
        return 0;
    }
    std::vector<std::thread> th;
    for (int c = 0; c < n_cams; ++c) th.emplace_back(one, c);
    for (auto &t : th) t.join();
    return 0;
}

float oracle_fast_atan2(float y, float x) { return oracle::fast_atan2_deg(y, x); }

}  // extern "C"
