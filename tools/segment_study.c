/*
 * segment_study.c -- design study (CPU, not product code): segment-parallel replay of a search pass.
 *
 * A pass over a ray's n cached samples at threshold t is split into K segments [s_k, s_k+1).  Lane k
 * runs the supersegment state machine (AccumulateVDI.comp:34-251) from s_k with a fresh state and
 * records the sample indices of its first M closes.  Lane k-1 runs on past s_k with the TRUE state
 * until its state meets lane k's: either it arrives at s_k not open (then lane k's run is exact from
 * s_k), or it closes at a sample where lane k closed too (one of k's recorded closes: after a close
 * at j the state depends on sample j alone).  From there lane k's closes are exact.  If no meeting
 * happens within lane k's recorded closes, lane k-1 goes on and tries lane k+1 at s_k+1.
 *
 * Reported per search pass (passes 2.. of the reference's binary search, VDIGenerator.comp:497-529,
 * full passes, no early exit): latency = max over lanes of the samples a lane replays, work = their
 * sum, both against n; and the count of the chained lanes must equal the unsegmented pass's.
 *
 * build: gcc -O3 -march=x86-64-v3 -std=gnu99 -fPIC -ffp-contract=off -shared -o /tmp/libsegstudy.so \
 *            tools/segment_study.c -lm   (driven by tools/segment_study.py)
 */
#include <stdio.h>
#include "../oracle/insitu_oracle.c"

#define MAXK 8
#define MAXM 8
#define CAP (1 << 14)

typedef struct {
    double rays, passes;              /* searched rays, search passes evaluated */
    double samples;                   /* sum of n over those passes */
    double lat[MAXK + 1];             /* sum over passes of the segmented latency, K = 1..MAXK */
    double work[MAXK + 1];            /* sum of the lanes' replayed samples */
    double unsynced[MAXK + 1];        /* lane boundaries never met within M recorded closes */
    double mismatch[MAXK + 1];        /* passes whose chained count differs (must stay 0) */
    double overlap_hist[MAXK + 1][8]; /* resync distance past s_k: 0, <=4, <=16, <=32, <=64, <=128, <=256, more */
} seg_out;

typedef struct {
    int nterm, open, steps_in;
    v4 curV;
} st_t;

/* one sample of the state machine; returns 1 when it closed at this sample (a decision >= t) */
static int step(st_t* s, const v4 x, float w, int last, float t, const v4 wfront, const v4 wback, float nw) {
    int closed = 0;
    if (!(x.x > -0.5f || last)) return 0;
    const int transparent = w <= 0.0f;
    if (s->open) {
        v4 jp = v4mix(wfront, wback, nw * (float)s->steps_in);
        float segLen = len4(jp.x - wfront.x, jp.y - wfront.y, jp.z - wfront.z, jp.w - wfront.w);
        float inva = 1.0f / s->curV.w;
        float ax = s->curV.x * inva, ay = s->curV.y * inva, az = s->curV.z * inva;
        float aw = adjust_opacity(s->curV.w, 1.0f / segLen);
        float bx = x.x * x.w, by = x.y * x.w, bz = x.z * x.w;
        float diff = len3(ax * aw - bx, ay * aw - by, az * aw - bz);
        if (diff >= t) {
            s->nterm++;
            s->open = 0;
            s->steps_in = 0;
            closed = 1;
        }
    }
    if (!s->open && !transparent) {
        s->open = 1;
        s->curV.x = s->curV.y = s->curV.z = s->curV.w = 0.0f;
    }
    if (s->open) {
        float tt = 1.0f - s->curV.w;
        s->curV.x = fmaf(tt * x.x, w, s->curV.x);
        s->curV.y = fmaf(tt * x.y, w, s->curV.y);
        s->curV.z = fmaf(tt * x.z, w, s->curV.z);
        s->curV.w = fmaf(tt, w, s->curV.w);
        s->steps_in++;
    }
    if (last && s->open) {
        s->nterm++;
        s->open = 0;
        s->steps_in = 0;
    }
    return closed;
}

static int bucket(int d) {
    return d <= 0 ? 0 : d <= 4 ? 1 : d <= 16 ? 2 : d <= 32 ? 3 : d <= 64 ? 4 : d <= 128 ? 5 : d <= 256 ? 6 : 7;
}

/* the segmented pass with K lanes, M recorded closes per lane: latency, work, chained count */
static void segmented(const v4* x, const float* w, const int* last, int n, float t, int K, int M, const v4 wf,
                      const v4 wb, float nw, int* lat, int* work, int* count, int* unsynced, seg_out* out) {
    int L = (n + K - 1) / K;
    L = (L + 3) & ~3;
    int s[MAXK + 1], rec[MAXK][MAXM], recn[MAXK][MAXM], nrec[MAXK], tot[MAXK], stopk[MAXK], tgt[MAXK], mk[MAXK];
    for (int k = 0; k <= K; ++k) s[k] = k * L < n ? k * L : n;
    /* lanes from the last to the first: a lane records the first M closes it makes before it stops (its
       predecessor checks them; the lanes run in parallel, a later lane ahead in sample position), and it
       stops where it meets a later lane (that lane's record is final by then) */
    *unsynced = 0;
    for (int k = K - 1; k >= 0; --k) {
        st_t st = {0, 0, 0, {0, 0, 0, 0}};
        int tg = k + 1, p = 0, i = s[k];
        tgt[k] = K;
        mk[k] = 0;
        nrec[k] = 0;
        for (; i < n; ++i) {
            while (tg < K && i >= s[tg] && p >= nrec[tg] && (nrec[tg] == M || stopk[tg] <= i)) {
                /* past tg's record (full, or tg stopped): tg can no longer be met, try the next lane */
                if (tg == k + 1) (*unsynced)++;
                tg++;
                p = 0;
            }
            if (tg < K && i == s[tg] && !st.open) {   /* arrives at s_tg not open: tg exact from there */
                tgt[k] = tg;
                mk[k] = 0;
                break;
            }
            const int closed = step(&st, x[i], w[i], last[i], t, wf, wb, nw);
            if (closed && nrec[k] < M) {   /* position and the count after it (a last-sample close included) */
                rec[k][nrec[k]] = i;
                recn[k][nrec[k]++] = st.nterm;
            }
            if (tg < K && i >= s[tg]) {
                while (p < nrec[tg] && rec[tg][p] < i) p++;
                if (closed && p < nrec[tg] && rec[tg][p] == i) {   /* a common close: tg exact after i */
                    tgt[k] = tg;
                    mk[k] = recn[tg][p];
                    i++;
                    break;
                }
            }
        }
        stopk[k] = i;
        tot[k] = st.nterm;
        if (tgt[k] < K) out->overlap_hist[K][bucket(i - s[tgt[k]])] += 1;
    }
    /* chain: lane 0, then the lane it met, ... */
    int c = 0, k = 0, m = 0, mx = 0, sum = 0;
    for (int j = 0; j < K; ++j) {
        const int len = stopk[j] - s[j];
        if (len > mx) mx = len;
        sum += len > 0 ? len : 0;
    }
    while (k < K) {
        /* lane k's closes from the start of its exact part: its total minus its first m closes */
        c += tot[k] - m;
        m = mk[k];
        k = tgt[k];
    }
    *lat = mx;
    *work = sum;
    *count = c;
}

int study_seg(const orc_brick* brick, const orc_transfer* tf, const orc_camera* cam, int W, int H, int S, int x0,
              int x1, int y0, int y1, int ystep, int M, seg_out* out) {
    vdi_job J;
    memset(&J, 0, sizeof J);
    J.b[0] = brick;
    J.nb = 1;
    J.tf = tf;
    J.cam = cam;
    orc_mat4_mul(cam->inv_view, cam->inv_proj, J.ipv);
    orc_mat4_mul(cam->proj, cam->view, J.pv);
    memset(out, 0, sizeof *out);
    const float nw = cam->nw;
    v4* xs = malloc(sizeof(v4) * CAP);
    float* ws = malloc(sizeof(float) * CAP);
    int* ls = malloc(sizeof(int) * CAP);
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
            int n = 0;
            float stp = tnear;
            v4 wprev = v4mix(wfront, wback, stp - nw);
            for (int i = 0; i < numSteps; ++i, stp += nw) {
                v4 wpos = v4mix(wfront, wback, stp);
                if (stp > n_ && stp < f_ && n < CAP) {
                    v4 xv = sample_volume(brick, tf, wpos);
                    xs[n] = xv;
                    ws[n] = adjust_opacity(xv.w, len4(wpos.x - wprev.x, wpos.y - wprev.y, wpos.z - wprev.z,
                                                      wpos.w - wprev.w));
                    ls[n] = (i == numSteps - 1);
                    n++;
                }
                wprev = wpos;
            }
            if (n == 0) continue;
            float low = 0.0f, high = 1.732f, mid = 0.0001f;
            int found = 0, first = 1, iter = 0, searched = 0;
            const int delta = (int)floorf(0.15f * (float)S);
            while (!found && iter < 64) {
                iter++;
                const float t = mid;
                st_t st = {0, 0, 0, {0, 0, 0, 0}};
                for (int i = 0; i < n; ++i) step(&st, xs[i], ws[i], ls[i], t, wfront, wback, nw);
                const int nterm = st.nterm;
                if (iter >= 2) {
                    searched = 1;
                    out->passes += 1;
                    out->samples += n;
                    for (int K = 1; K <= MAXK; ++K) {
                        int lat, work, cnt, uns;
                        segmented(xs, ws, ls, n, t, K, M, wfront, wback, nw, &lat, &work, &cnt, &uns, out);
                        out->lat[K] += lat;
                        out->work[K] += work;
                        out->unsynced[K] += uns;
                        if (cnt != nterm) {
                            out->mismatch[K] += 1;
                            if (K == 2 && getenv("SEG_DEBUG") && out->mismatch[K] < 4) {
                                fprintf(stderr, "mismatch n=%d t=%g nterm=%d cnt=%d\n", n, t, nterm, cnt);
                                st_t a = {0, 0, 0, {0, 0, 0, 0}};
                                int L = ((n + 1) / 2 + 3) & ~3;
                                fprintf(stderr, "true closes:");
                                for (int i = 0; i < n; ++i) if (step(&a, xs[i], ws[i], ls[i], t, wfront, wback, nw)) fprintf(stderr, " %d", i);
                                fprintf(stderr, "\nfresh from %d:", L);
                                st_t b = {0, 0, 0, {0, 0, 0, 0}};
                                for (int i = L; i < n; ++i) if (step(&b, xs[i], ws[i], ls[i], t, wfront, wback, nw)) fprintf(stderr, " %d", i);
                                fprintf(stderr, "\n true total %d fresh total %d\n", a.nterm, b.nterm);
                            }
                        }
                    }
                }
                if (fabsf(high - low) < 0.000001f) {
                    found = 1;
                    break;
                } else if (nterm > S) {
                    low = mid;
                } else if (nterm < S - delta) {
                    high = mid;
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
            out->rays += searched;
        }
    free(xs);
    free(ws);
    free(ls);
    return 0;
}
