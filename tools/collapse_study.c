/*
 * collapse_study.c -- design study (CPU, not product code): can the rays whose threshold search runs to
 * the interval collapse (VDIGenerator.comp:497-529: |high - low| < 1e-6, ~24 passes, the critical path
 * of a one-brick search) be told apart after pass 1 and the four spine levels the sampling kernel runs?
 * Per searched ray: n, the counts at 1e-4 and at the spine thresholds 0.866 / 0.433 / 0.217 / 0.108,
 * and the passes of the whole search.  Reuses the oracle by inclusion; driven by tools/collapse_study.py.
 */
#include "../oracle/insitu_oracle.c"

typedef struct { int n, c[5], passes, l1_implied; } cray;

static float g_lo, g_hi;   /* segmentation interval of the last cpass (squared differences) */
static int cpass(const v4* x, const float* w, const int* last, int n, float t, int S, int early,
                 const v4 wfront, const v4 wback, float nw) {
    int nterm = 0, open = 0, steps_in = 0;
    g_lo = 0.0f; g_hi = INFINITY;
    v4 curV = {0, 0, 0, 0};
    for (int i = 0; i < n; ++i) {
        if (!(x[i].x > -0.5f || last[i])) continue;
        const int transparent = w[i] <= 0.0f;
        if (open) {
            v4 jp = v4mix(wfront, wback, nw * (float)steps_in);
            float segLen = len4(jp.x - wfront.x, jp.y - wfront.y, jp.z - wfront.z, jp.w - wfront.w);
            float inva = 1.0f / curV.w;
            float ax = curV.x * inva, ay = curV.y * inva, az = curV.z * inva;
            float aw = adjust_opacity(curV.w, 1.0f / segLen);
            float bx = x[i].x * x[i].w, by = x[i].y * x[i].w, bz = x[i].z * x[i].w;
            float diff = len3(ax * aw - bx, ay * aw - by, az * aw - bz);
            if (diff >= t) { nterm++; open = 0; steps_in = 0; if (diff * diff < g_hi) g_hi = diff * diff; }
            else if (diff * diff > g_lo) g_lo = diff * diff;
        }
        if (!open && !transparent) { open = 1; curV.x = curV.y = curV.z = curV.w = 0.0f; }
        if (open) {
            float tt = 1.0f - curV.w;
            curV.x = fmaf(tt * x[i].x, w[i], curV.x);
            curV.y = fmaf(tt * x[i].y, w[i], curV.y);
            curV.z = fmaf(tt * x[i].z, w[i], curV.z);
            curV.w = fmaf(tt, w[i], curV.w);
            steps_in++;
        }
        if (last[i] && open) { nterm++; open = 0; steps_in = 0; }
        if (early && nterm > S) return nterm;
    }
    return nterm;
}

int study_collapse(const orc_brick* brick, const orc_transfer* tf, const orc_camera* cam, int W, int H, int S,
                   int x0, int x1, int y0, int y1, int ystep, cray* out, int cap_rays) {
    float ipv[16];
    orc_mat4_mul(cam->inv_view, cam->inv_proj, ipv);
    const float nw = cam->nw;
    int cap = 1 << 14, nr = 0;
    v4* xs = malloc(sizeof(v4) * cap);
    float* ws = malloc(sizeof(float) * cap);
    int* ls = malloc(sizeof(int) * cap);
    for (int gy = y0; gy < y1; gy += ystep)
        for (int gx = x0; gx < x1; ++gx) {
            float uvx = fmaf((float)gx / (float)W, 2.0f, -1.0f), uvy = fmaf((float)gy / (float)H, 2.0f, -1.0f);
            v4 front = {uvx, uvy, -1.0f, 1.0f}, back = {uvx, uvy, 1.0f, 1.0f};
            v4 wfront = persp_div(mat_vec(ipv, front)), wback = persp_div(mat_vec(ipv, back));
            float n_, f_;
            intersect_bbox(brick, wfront, wback, &n_, &f_);
            f_ = gmin(cam->tmax, f_);
            if (!(n_ < f_)) continue;
            float tnear = gmin(1.0f, gmax(0.0f, n_)), tfar = gmax(0.0f, f_);
            if (!(tnear < tfar)) continue;
            int numSteps = (int)truncf((tfar - tnear) / nw);
            int n = 0;
            float step = tnear;
            v4 wprev = v4mix(wfront, wback, step - nw);
            for (int i = 0; i < numSteps; ++i, step += nw) {
                v4 wpos = v4mix(wfront, wback, step);
                if (step > n_ && step < f_ && n < cap) {
                    v4 x = sample_volume(brick, tf, wpos);
                    xs[n] = x;
                    ws[n] = adjust_opacity(x.w, len4(wpos.x - wprev.x, wpos.y - wprev.y, wpos.z - wprev.z, wpos.w - wprev.w));
                    ls[n] = (i == numSteps - 1);
                    n++;
                }
                wprev = wpos;
            }
            if (n == 0 || nr >= cap_rays) continue;
            cray r = {n, {0}, 0, 0};
            {   /* the spine's level 2 (0.433): does its interval hold level 1's threshold (0.866)? */
                const float t2 = ((0.0001f + 1.732f) / 2.0f + 0.0001f) / 2.0f, t1 = (0.0001f + 1.732f) / 2.0f;
                (void)cpass(xs, ws, ls, n, t2, S, 1, wfront, wback, nw);
                r.l1_implied = (g_lo < t1 * t1 && t1 * t1 <= g_hi) ? 1 : 0;
            }
            float low = 0.0f, high = 1.732f, mid = 0.0001f;
            int iter = 0, first = 1;
            const int delta = (int)floorf(0.15f * (float)S);
            while (iter < 64) {
                iter++;
                int nterm = cpass(xs, ws, ls, n, mid, S, 1, wfront, wback, nw);
                if (iter <= 5) r.c[iter - 1] = nterm;
                if (fabsf(high - low) < 0.000001f) break;
                else if (nterm > S) low = mid;
                else if (nterm < S - delta) high = mid;
                else break;
                if (first) { first = 0; if (nterm < S) break; }
                mid = (low + high) / 2.0f;
            }
            r.passes = iter;
            if (r.c[0] > S) out[nr++] = r;   /* searched rays only */
        }
    free(xs); free(ws); free(ls);
    return nr;
}
