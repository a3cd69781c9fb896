/*
 * bound_study.c -- design study (CPU, not product code): how often would a CHEAP bound decide a
 * supersegment test `diff >= t` (AccumulateVDI.comp:50-74) without the full estimate?
 *
 * diff = |c*aw - y| with c = curV.rgb / curV.a (a weighted mean of sample colours, |c_i| <= C),
 * aw = 1 - (1 - A)^(1/L) (A = curV.a, L = segLen) and y = x.rgb * x.a.  Bernoulli gives
 * aw <= A * max(1, 1/L), so diff_i <= C * A * max(1, 1/L) + |y_i| for every channel: when that upper
 * bound is below t, the test certainly fails ("no close") with a handful of operations.  Counted over
 * every decision of every pass of the search (the passes the kernels run, early exit at nterm > S),
 * split into pass 1 (t = 1e-4) and the later passes; the true 1/L is used (optimistic).
 *
 * Reuses the oracle's sampling code by inclusion (oracle/insitu_oracle.c, single-volume rays);
 * driven by tools/bound_study.py.
 */
#include "../oracle/insitu_oracle.c"

typedef struct {
    double dec[2], nocl_bound[2], close[2], hist[2][16];   /* [0] pass 1, [1] later passes */
    double rays;
    double steps_hist[2][8];   /* decisions by steps_in: 1,2-4,5-8,9-16,17-32,33-64,65-128,>128 */
    double max_relerr[8];      /* max |1/L_crude - 1/L| * L over the same steps classes (L_crude = t * |wb - wf|) */
    double spine_dec[4], spine_bound[4];   /* decisions at the spine thresholds 0.866/0.433/0.217/0.108, and those the bound settles */
} bstudy_out;

static int bpass(const v4* x, const float* w, const int* last, int n, float t, int S, int early, float C,
                 const v4 wfront, const v4 wback, float nw, bstudy_out* o, int k) {
    int nterm = 0, open = 0, steps_in = 0;
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
            const float il = 1.0f / segLen, m = curV.w * (il > 1.0f ? il : 1.0f) * C;
            const float ub = sqrtf((m + fabsf(bx)) * (m + fabsf(bx)) + (m + fabsf(by)) * (m + fabsf(by)) +
                                   (m + fabsf(bz)) * (m + fabsf(bz)));
            o->dec[k] += 1;
            {
                int c = steps_in <= 1 ? 0 : (steps_in <= 4 ? 1 : (steps_in <= 8 ? 2 : (steps_in <= 16 ? 3 : (steps_in <= 32 ? 4 : (steps_in <= 64 ? 5 : (steps_in <= 128 ? 6 : 7))))));
                o->steps_hist[k][c] += 1;
                double D = sqrt((double)(wback.x - wfront.x) * (wback.x - wfront.x) + (double)(wback.y - wfront.y) * (wback.y - wfront.y) +
                                (double)(wback.z - wfront.z) * (wback.z - wfront.z) + (double)(wback.w - wfront.w) * (wback.w - wfront.w));
                double Lc = (double)(nw * (float)steps_in) * D;
                double re = fabs(Lc / (double)segLen - 1.0);
                if (re > o->max_relerr[c]) o->max_relerr[c] = re;
            }
            if (ub < t) o->nocl_bound[k] += 1;
            int hb = diff > 0 ? (int)floorf(log10f(diff / t)) + 8 : 0;
            o->hist[k][hb < 0 ? 0 : (hb > 15 ? 15 : hb)] += 1;
            if (diff >= t) {
                o->close[k] += 1;
                nterm++;
                open = 0;
                steps_in = 0;
            }
        }
        if (!open && !transparent) {
            open = 1;
            curV.x = curV.y = curV.z = curV.w = 0.0f;
        }
        if (open) {
            float tt = 1.0f - curV.w;
            curV.x = fmaf(tt * x[i].x, w[i], curV.x);
            curV.y = fmaf(tt * x[i].y, w[i], curV.y);
            curV.z = fmaf(tt * x[i].z, w[i], curV.z);
            curV.w = fmaf(tt, w[i], curV.w);
            steps_in++;
        }
        if (last[i] && open) {
            nterm++;
            open = 0;
            steps_in = 0;
        }
        if (early && nterm > S) return nterm;
    }
    return nterm;
}

int study_bound(const orc_brick* brick, const orc_transfer* tf, const orc_camera* cam, int W, int H, int S, int x0,
                int x1, int y0, int y1, int ystep, float C, bstudy_out* out) {
    float ipv[16];
    orc_mat4_mul(cam->inv_view, cam->inv_proj, ipv);
    memset(out, 0, sizeof *out);
    const float nw = cam->nw;
    int cap = 1 << 14;
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
                    ws[n] = adjust_opacity(x.w, len4(wpos.x - wprev.x, wpos.y - wprev.y, wpos.z - wprev.z,
                                                     wpos.w - wprev.w));
                    ls[n] = (i == numSteps - 1);
                    n++;
                }
                wprev = wpos;
            }
            if (n == 0) continue;
            out->rays += 1;
            {
                bstudy_out tmp;
                float tl = 0.0001f, th = 1.732f, tm = (tl + th) / 2.0f;
                for (int l = 0; l < 4; ++l) {
                    memset(&tmp, 0, sizeof tmp);
                    (void)bpass(xs, ws, ls, n, tm, S, 1, C, wfront, wback, nw, &tmp, 0);
                    out->spine_dec[l] += tmp.dec[0];
                    out->spine_bound[l] += tmp.nocl_bound[0];
                    th = tm;
                    tm = (tl + th) / 2.0f;
                }
            }
            float low = 0.0f, high = 1.732f, mid = 0.0001f;
            int iter = 0, first = 1;
            const int delta = (int)floorf(0.15f * (float)S);
            while (iter < 64) {
                iter++;
                int nterm = bpass(xs, ws, ls, n, mid, S, iter >= 2, C, wfront, wback, nw, out, iter >= 2);
                if (fabsf(high - low) < 0.000001f) break;
                else if (nterm > S) low = mid;
                else if (nterm < S - delta) high = mid;
                else break;
                if (first) {
                    first = 0;
                    if (nterm < S) break;
                }
                mid = (low + high) / 2.0f;
            }
        }
    free(xs);
    free(ws);
    free(ls);
    return 0;
}
