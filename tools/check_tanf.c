/* Check that the glibc tanf restatement (fdlibm __kernel_tanf after a double-precision reduction; same
 * constants and operation order as openmavis_amd/csrc/omv_device.h::glibc_tanf, used by
 * KannalaBrandt8::unproject's std::tan(theta)) is bit-identical to the host libm on every float with
 * |x| < 120 (2.2e9 inputs, 0 mismatches against glibc 2.35; the Newton-refined theta stays < pi/2).
 * gcc -O2 -ffp-contract=off tools/check_tanf.c -lm && ./a.out */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static inline uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float bitsf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static const float T[] = {3.3333334327e-01f, 1.3333334029e-01f, 5.3968254477e-02f, 2.1869488060e-02f,
                          8.8632395491e-03f, 3.5920790397e-03f, 1.4562094584e-03f, 5.8804126456e-04f,
                          2.4646313977e-04f, 7.8179444245e-05f, 7.1407252108e-05f, -1.8558637748e-05f,
                          2.5907305826e-05f};
static const float pio4 = 7.8539812565e-01f, pio4lo = 3.7748947079e-08f;
static float kernel_tanf(float x, float y, int iy) {
    float z, r, v, w, s;
    int32_t hx = (int32_t)fbits(x), ix = hx & 0x7fffffff;
    if (ix < 0x39000000) {   /* |x| < 2**-13 */
        if ((int)x == 0) {
            if ((ix | (iy + 1)) == 0) return 1.0f / fabsf(x);
            else if (iy == 1) return x;
            else return -1.0f / x;
        }
    }
    if (ix >= 0x3f2ca140) {   /* |x| >= 0.6744 */
        if (hx < 0) { x = -x; y = -y; }
        z = pio4 - x;
        w = pio4lo - y;
        x = z + w;
        y = 0.0f;
        if (fabsf(x) < 0x1p-13f) return (1 - ((hx >> 30) & 2)) * iy * (1.0f - 2 * iy * x);
    }
    z = x * x;
    w = z * z;
    r = T[1] + w * (T[3] + w * (T[5] + w * (T[7] + w * (T[9] + w * T[11]))));
    v = z * (T[2] + w * (T[4] + w * (T[6] + w * (T[8] + w * (T[10] + w * T[12])))));
    s = z * x;
    r = y + z * (s * (r + v) + y);
    r += T[0] * s;
    w = x + r;
    if (ix >= 0x3f2ca140) {
        v = (float)iy;
        return (float)(1 - ((hx >> 30) & 2)) * (v - 2.0f * (x - (w * w / (w + v) - r)));
    }
    if (iy == 1) return w;
    {
        float a, t;
        z = w;
        z = bitsf(fbits(z) & 0xfffff000);
        v = r - (z - x);
        t = a = -1.0f / w;
        t = bitsf(fbits(t) & 0xfffff000);
        s = 1.0f + t * z;
        return t + a * (s + t * v);
    }
}
/* glibc's tanf reduces pi/4 < |x| < 120 in double: n = nearbyint(x 2/pi), r = x - n pi/2, then
 * y = (float)r, (float)(r - y).  (An fdlibm float-only __ieee754_rem_pio2f differs from glibc 2.35 on
 * 1034 inputs below 3pi/4; this form matches all of them.) */
float my_tanf(float x) {
    int32_t hx = (int32_t)fbits(x), ix = hx & 0x7fffffff;
    if (ix <= 0x3f490fda) return kernel_tanf(x, 0.0f, 1);
    const double xd = (double)x, nd = nearbyint(xd * 0.6366197723675814);
    const int n = (int)nd;
    const double r = xd - nd * 1.5707963267948966;
    const float y0 = (float)r, y1 = (float)(r - (double)y0);
    return kernel_tanf(y0, y1, 1 - ((n & 1) << 1));
}
int main(void) {
    long n = 0, bad = 0;
    for (uint32_t u = 0; u < 0x42f00000u; ++u) {   /* |x| < 120 */
        const float x = bitsf(u);
        for (int sg = 0; sg < 2; ++sg) {
            const float xx = sg ? -x : x;
            const float g = tanf(xx), m = my_tanf(xx);
            ++n;
            if (fbits(g) != fbits(m)) {
                if (bad < 10) printf("x=%a glibc=%a mine=%a\n", xx, g, m);
                ++bad;
            }
        }
    }
    printf("checked %ld floats with |x| < 120: %ld mismatches\n", n, bad);
    return bad != 0;
}
