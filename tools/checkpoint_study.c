/*
 * checkpoint_study.c -- design study (CPU, not product code): how much replay work would the
 * threshold search save if a search pass could resume from a saved state of an earlier pass?
 *
 * The search kernel replays a ray's cached samples once per binary-search pass.  Two passes at
 * thresholds t and tX make identical decisions -- hence reach identical states -- up to the first
 * sample where pass X tested a difference d with (d >= tX) != (d >= t).  A pass at t could therefore
 * start from X's state at (or before) that sample.  X = the passes at the current `low` and `high`
 * thresholds (the bracket of the binary search, VDIGenerator.comp:497-529).  States saved every K
 * cache samples: the resume point is rounded down to a multiple of K.
 *
 * Counted in cache samples replayed by the search passes (every pass after the first, the write
 * pass excluded), early-exit at nterm > S as the kernel does.  Baseline = what the kernel does now,
 * including its whole-pass skip (a pass with no divergence from the low or high pass costs 0).
 *
 * Reuses the oracle's sampling code by inclusion (oracle/insitu_oracle.c, single-volume rays).
 * build: gcc -O3 -march=x86-64-v3 -std=c99 -fPIC -ffp-contract=off -fopenmp -shared \
 *            -o /tmp/libckstudy.so tools/checkpoint_study.c -lm
 * driven by tools/checkpoint_study.py.
 */
#include "../oracle/insitu_oracle.c"

#define KMAX 4
static const int KS[KMAX] = {1, 16, 32, 64};

typedef struct {
    double rays, passes_hist[65];
    double base, ck[KMAX], search_passes, skipped_base;
    double samples;   /* total cache samples over searched rays */
    double real_by_passes[65];   /* replayed (non-skipped) search passes, by the ray's total passes */
    double left_run[65];         /* searched rays whose first k search decisions (after pass 1) went left (high = mid) */
    double dec[4][4][3];         /* decisions after the 4-level spine: [prev2][prev1][next], L=0 R=1 F=2, 3 = none */
    double base_by_passes[65];   /* replayed samples of the search passes, by the ray's total passes */
    double ck1_by_passes[65];    /* ... resuming from per-sample states of the low/high passes */
    double ck16_by_passes[65];   /* ... from states every 16 samples */
    double write_samples;        /* samples of separate write passes (accepted before pass 8, INSITU_SPEC_FROM) */
    double write_samples_rec;    /* ... of those whose accepted pass was a replayed pass with <= S closes */
} study_out;

/* one pass over the recorded samples at threshold t; fills d[i] (tested difference, or -1 when no
 * test happened at sample i) and returns nterm; *stop = samples replayed (early exit at nterm > S
 * when early != 0) */
static int pass(const v4* x, const float* w, const int* last, int n, const float* seglen_tab, float t, int S,
                int early, float* d, int* stop, const v4 wfront, const v4 wback, float nw) {
    int nterm = 0, open = 0, steps_in = 0;
    v4 curV = {0, 0, 0, 0};
    (void)seglen_tab;
    for (int i = 0; i < n; ++i) {
        d[i] = -1.0f;
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
            d[i] = diff;
            if (diff >= t) {
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
        if (early && nterm > S) {
            *stop = i + 1;
            return nterm;
        }
    }
    *stop = n;
    return nterm;
}

/* first sample where a pass at t decides differently from the recorded pass (dX, tX) */
static int divergence(const float* dX, int nX, float tX, float t) {
    for (int i = 0; i < nX; ++i)
        if (dX[i] >= 0.0f && ((dX[i] >= tX) != (dX[i] >= t))) return i;
    return nX;
}

int study_vdi(const orc_brick* brick, const orc_transfer* tf, const orc_camera* cam, int W, int H, int S, int x0,
              int x1, int y0, int y1, int ystep, study_out* out) {
    vdi_job J;
    memset(&J, 0, sizeof J);
    J.b[0] = brick;
    J.nb = 1;
    J.tf = tf;
    J.cam = cam;
    orc_mat4_mul(cam->inv_view, cam->inv_proj, J.ipv);
    orc_mat4_mul(cam->proj, cam->view, J.pv);
    J.W = W;
    J.H = H;
    J.S = S;
    memset(out, 0, sizeof *out);
    const float nw = cam->nw;
    int cap = 1 << 14;
    v4* xs = malloc(sizeof(v4) * cap);
    float* ws = malloc(sizeof(float) * cap);
    int* ls = malloc(sizeof(int) * cap);
    float* dcur = malloc(sizeof(float) * cap);
    float* dlow = malloc(sizeof(float) * cap);
    float* dhigh = malloc(sizeof(float) * cap);
    for (int gy = y0; gy < y1; gy += ystep)
        for (int gx = x0; gx < x1; ++gx) {
            float uvx = fmaf((float)gx / (float)W, 2.0f, -1.0f), uvy = fmaf((float)gy / (float)H, 2.0f, -1.0f);
            v4 front = {uvx, uvy, -1.0f, 1.0f}, back = {uvx, uvy, 1.0f, 1.0f};
            v4 wfront = persp_div(mat_vec(J.ipv, front)), wback = persp_div(mat_vec(J.ipv, back));
            float n_, f_;
            intersect_bbox(brick, wfront, wback, &n_, &f_);
            f_ = gmin(cam->tmax, f_);
            if (!(n_ < f_)) continue;
            float tnear = gmin(1.0f, gmax(0.0f, n_)), tfar = gmax(0.0f, f_);
            if (!(tnear < tfar)) continue;
            int numSteps = (int)truncf((tfar - tnear) / nw);
            /* record the in-brick samples (the cache entries) */
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
            /* the search (VG:380-529) */
            float low = 0.0f, high = 1.732f, mid = 0.0001f;
            int found = 0, first = 1, iter = 0, have_low = 0, have_high = 0, stop;
            const int delta = (int)floorf(0.15f * (float)S);
            int nlow = 0, nhigh = 0;
            int searched = 0, real = 0, left = 0, still_left = 1, p1 = 3, p2 = 3;
            double ray_base = 0.0, ray_ck1 = 0.0, ray_ck16 = 0.0;
            while (!found && iter < 64) {
                iter++;
                const float t = mid;
                /* pass 1 (sampling kernel) runs the whole ray; search passes stop at nterm > S */
                int nterm = pass(xs, ws, ls, n, NULL, t, S, iter >= 2, dcur, &stop, wfront, wback, nw);
                if (iter >= 2) {
                    int dl = have_low ? divergence(dlow, nlow, low, t) : 0;
                    int dh = have_high ? divergence(dhigh, nhigh, high, t) : 0;
                    /* whole-pass skip (free_walk): no divergence over the recorded part of the low pass
                       (its outcome, count > S, was decided there) or over the whole high pass */
                    int skip = (have_low && dl >= nlow) || (have_high && dh >= nhigh);
                    out->search_passes += 1;
                    if (skip) {
                        out->skipped_base += 1;
                    } else {
                        real++;
                        out->base += stop;
                        ray_base += stop;
                        int r = dl > dh ? dl : dh;
                        for (int k = 0; k < KMAX; ++k) {
                            int rk = (r / KS[k]) * KS[k];
                            if (rk > stop) rk = stop;
                            out->ck[k] += stop - rk;
                            if (KS[k] == 1) ray_ck1 += stop - rk;
                            if (KS[k] == 16) ray_ck16 += stop - rk;
                        }
                    }
                    searched = 1;
                }
                if (iter >= 2 && !(nterm < S - delta)) still_left = 0;
                if (iter >= 6) {
                    const int dcur = (fabsf(high - low) < 0.000001f) ? 2 : (nterm > S ? 1 : (nterm < S - delta ? 0 : 2));
                    out->dec[p2][p1][dcur] += 1;
                    p2 = p1;
                    p1 = dcur;
                }
                if (fabsf(high - low) < 0.000001f) {
                    found = 1;
                    break;
                } else if (nterm > S) {
                    low = mid;
                    memcpy(dlow, dcur, sizeof(float) * stop);
                    nlow = stop;
                    have_low = 1;
                } else if (nterm < S - delta) {
                    if (iter >= 2 && still_left) left++;
                    high = mid;
                    memcpy(dhigh, dcur, sizeof(float) * n);
                    nhigh = n;
                    have_high = 1;
                } else {
                    found = 1;
                    break;
                }
                if (first) {
                    first = 0;
                    if (nterm < S) {
                        found = 1;
                        break;
                    }
                }
                mid = (low + high) / 2.0f;
            }
            /* the write pass: separate unless the accepted pass is a search pass numbered >= 8 (it stored) */
            {
                const int accepted_replayed = found && iter >= 2 && !(fabsf(high - low) < 0.000001f);
                if (!(accepted_replayed && iter >= 8)) {
                    out->write_samples += n;
                    if (accepted_replayed) out->write_samples_rec += n;
                }
            }
            out->rays += 1;
            out->passes_hist[iter + 1 > 64 ? 64 : iter + 1] += 1;   /* + the write pass */
            out->real_by_passes[iter + 1 > 64 ? 64 : iter + 1] += real;
            out->base_by_passes[iter + 1 > 64 ? 64 : iter + 1] += ray_base;
            out->ck1_by_passes[iter + 1 > 64 ? 64 : iter + 1] += ray_ck1;
            out->ck16_by_passes[iter + 1 > 64 ? 64 : iter + 1] += ray_ck16;
            if (searched) { out->samples += n; out->left_run[left > 64 ? 64 : left] += 1; }
        }
    free(xs);
    free(ws);
    free(ls);
    free(dcur);
    free(dlow);
    free(dhigh);
    return 0;
}
