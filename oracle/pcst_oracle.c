/*
 * pcst_oracle.c -- CPU restatement of the reference's geometry / index work.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker.
 * The product path (pointcloud_style_transfer_amd) never links or calls it.
 *
 * Pinned against golden vectors produced by running the reference itself
 * (tests/golden/gen_golden.py).  Compiled with -ffp-contract=off so every
 * float operation below is the single IEEE operation it is written as; the
 * fused multiply-adds the reference's MKL K=3 matmul performs are spelled
 * out with fmaf().
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* Squared norm, unfused ((x0^2 + x1^2) + x2^2)  (pointnet2_encoder.py:13-14, Q2). */
static inline float sqnorm3(const float* p) {
    float a = p[0] * p[0];
    float b = p[1] * p[1];
    float c = p[2] * p[2];
    return (a + b) + c;
}

/* dot via the K=3 sgemm FMA chain fma(a2,b2,fma(a1,b1,a0*b0))  (Q1). */
static inline float dot3_fma(const float* a, const float* b) {
    return fmaf(a[2], b[2], fmaf(a[1], b[1], a[0] * b[0]));
}

/* square_distance (pointnet2_encoder.py:8-15): ((-2*dot) + |src|^2) + |dst|^2. */
void orc_square_distance(const float* src, const float* dst, int64_t B, int64_t S, int64_t N,
                         float* out) {
    for (int64_t b = 0; b < B; ++b)
        for (int64_t s = 0; s < S; ++s) {
            const float* a = src + (b * S + s) * 3;
            float na = sqnorm3(a);
            for (int64_t n = 0; n < N; ++n) {
                const float* q = dst + (b * N + n) * 3;
                float d = -2.0f * dot3_fma(a, q);
                d += na;
                d += sqnorm3(q);
                out[(b * S + s) * N + n] = d;
            }
        }
}

/* farthest_point_sample (pointnet2_encoder.py:30-45).
 * distance init 1e10; per iteration: dist = ((dx^2+dy^2)+dz^2) unfused,
 * distance = dist where dist < distance (strict), next = argmax, lowest index on ties (Q3). */
void orc_fps(const float* xyz, int64_t B, int64_t N, int64_t npoint, const int64_t* start,
             int64_t* out) {
    float* dist = (float*)malloc(sizeof(float) * (size_t)N);
    for (int64_t b = 0; b < B; ++b) {
        const float* P = xyz + b * N * 3;
        for (int64_t n = 0; n < N; ++n) dist[n] = 1e10f;
        int64_t far = start[b];
        for (int64_t i = 0; i < npoint; ++i) {
            out[b * npoint + i] = far;
            float cx = P[far * 3 + 0], cy = P[far * 3 + 1], cz = P[far * 3 + 2];
            float best = -1.0f;
            int64_t besti = 0;
            for (int64_t n = 0; n < N; ++n) {
                float dx = P[n * 3 + 0] - cx, dy = P[n * 3 + 1] - cy, dz = P[n * 3 + 2] - cz;
                float xx = dx * dx, yy = dy * dy, zz = dz * dz;
                float d = (xx + yy) + zz;
                if (d < dist[n]) dist[n] = d;
                if (dist[n] > best) { best = dist[n]; besti = n; }
            }
            far = besti;
        }
    }
    free(dist);
}

/* query_ball_point (pointnet2_encoder.py:47-59): first nsample indices j (ascending) with
 * !(D[s,j] > r^2), D from square_distance(new_xyz, xyz), r^2 rounded to fp32 (Q4);
 * missing slots padded with the first found; if none found the value is N. */
void orc_ball_query(double radius, int64_t nsample, const float* xyz, const float* new_xyz,
                    int64_t B, int64_t N, int64_t S, int64_t* out) {
    float r2 = (float)(radius * radius);
    for (int64_t b = 0; b < B; ++b)
        for (int64_t s = 0; s < S; ++s) {
            const float* a = new_xyz + (b * S + s) * 3;
            float na = sqnorm3(a);
            int64_t* o = out + (b * S + s) * nsample;
            int64_t cnt = 0;
            for (int64_t n = 0; n < N && cnt < nsample; ++n) {
                const float* q = xyz + (b * N + n) * 3;
                float d = -2.0f * dot3_fma(a, q);
                d += na;
                d += sqnorm3(q);
                if (!(d > r2)) o[cnt++] = n;
            }
            int64_t first = cnt > 0 ? o[0] : N;
            for (int64_t k = cnt; k < nsample; ++k) o[k] = first;
        }
}

/* ---- voxel statistics of HierarchicalProcessor._voxel_grid_downsample_torch ----------------
 * (diffusion_model.py:78-97) for ONE cloud:
 *   vs = float(pow(double(f32(prod(range)) / target), 1/3)) * 1.2f   (0-d tensor pow runs in
 *        double: verified bit-exact in the survey container), range < 1e-6 -> 1, vs < 1e-6 -> 1e-3
 *   v  = int32(floor((p - min) / vs))
 *   h  = (vx*73856093) ^ (vy*19349663) ^ (vz*83492791)    int32 wrap-around  (Q5)
 *   unique(h) ascending (signed), rep_k = trunc(f32(sum idx) / f32(count))   (Q6)
 * Writes reps in ascending-hash order; returns U.  Also returns the voxel size and hashes. */
typedef struct { int32_t key; int32_t idx; } kv_t;

static int cmp_kv(const void* a, const void* b) {
    const kv_t* x = (const kv_t*)a;
    const kv_t* y = (const kv_t*)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->idx < y->idx ? -1 : (x->idx > y->idx);
}

static inline int32_t wrap_mul(int32_t a, int32_t m) {
    return (int32_t)((uint32_t)a * (uint32_t)m);
}

int64_t orc_voxel_reps(const float* pts, int64_t N, int64_t target, int64_t* reps,
                       int32_t* hash_out, float* vs_out) {
    float mn[3], mx[3], rg[3];
    for (int c = 0; c < 3; ++c) { mn[c] = pts[c]; mx[c] = pts[c]; }
    for (int64_t n = 1; n < N; ++n)
        for (int c = 0; c < 3; ++c) {
            float v = pts[n * 3 + c];
            if (v < mn[c]) mn[c] = v;
            if (v > mx[c]) mx[c] = v;
        }
    for (int c = 0; c < 3; ++c) {
        rg[c] = mx[c] - mn[c];
        if (rg[c] < 1e-6f) rg[c] = 1.0f;
    }
    float prod = (rg[0] * rg[1]) * rg[2];
    float q = prod / (float)target;
    float vs = (float)pow((double)q, 1.0 / 3.0);
    vs = vs * 1.2f;
    if (vs < 1e-6f) vs = 1e-3f;
    if (vs_out) *vs_out = vs;
    kv_t* kv = (kv_t*)malloc(sizeof(kv_t) * (size_t)N);
    for (int64_t n = 0; n < N; ++n) {
        int32_t v[3];
        for (int c = 0; c < 3; ++c) v[c] = (int32_t)floorf((pts[n * 3 + c] - mn[c]) / vs);
        int32_t h = wrap_mul(v[0], 73856093) ^ wrap_mul(v[1], 19349663) ^ wrap_mul(v[2], 83492791);
        kv[n].key = h;
        kv[n].idx = (int32_t)n;
        if (hash_out) hash_out[n] = h;
    }
    qsort(kv, (size_t)N, sizeof(kv_t), cmp_kv);
    int64_t U = 0;
    int64_t i = 0;
    while (i < N) {
        int64_t j = i;
        int64_t sum = 0;
        while (j < N && kv[j].key == kv[i].key) { sum += kv[j].idx; ++j; }
        int64_t cnt = j - i;
        reps[U++] = (int64_t)((float)sum / (float)cnt);
        i = j;
    }
    free(kv);
    return U;
}

/* ---- HierarchicalProcessor.upsample_knn core (diffusion_model.py:127-153) ------------------
 * For each query (float32 -> float64) find the k nearest refs by float64 rdist
 * ((dx*dx + dy*dy) + dz*dz) (sklearn KD-tree, euclidean rdist), ascending, ties -> lower ref
 * position; w = 1/(sqrt(rdist)+1e-8); w /= ((w0+w1)+w2); out = sum_k vals[nbr_k] * w_k
 * (float64, sequential), rounded to float32.  Brute force, parallel over queries. */
void orc_knn_interp(const float* refs, const float* vals, int64_t R, const float* queries,
                    int64_t Q, int64_t k, float* out, int64_t* nbr_out) {
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t q = 0; q < Q; ++q) {
        double qx = queries[q * 3 + 0], qy = queries[q * 3 + 1], qz = queries[q * 3 + 2];
        double bd[3] = {INFINITY, INFINITY, INFINITY};
        int64_t bi[3] = {-1, -1, -1};
        for (int64_t r = 0; r < R; ++r) {
            double dx = qx - (double)refs[r * 3 + 0];
            double dy = qy - (double)refs[r * 3 + 1];
            double dz = qz - (double)refs[r * 3 + 2];
            double xx = dx * dx, yy = dy * dy, zz = dz * dz;
            double d = (xx + yy) + zz;
            if (d < bd[k - 1]) {
                int64_t p = k - 1;
                while (p > 0 && d < bd[p - 1]) { bd[p] = bd[p - 1]; bi[p] = bi[p - 1]; --p; }
                bd[p] = d;
                bi[p] = r;
            }
        }
        double w[3], ws = 0.0;
        for (int64_t j = 0; j < k; ++j) {
            double dist = sqrt(bd[j]);
            w[j] = 1.0 / (dist + 1e-8);
        }
        for (int64_t j = 0; j < k; ++j) ws = j == 0 ? w[0] : ws + w[j];
        for (int64_t j = 0; j < k; ++j) w[j] = w[j] / ws;
        for (int c = 0; c < 3; ++c) {
            double acc = 0.0;
            for (int64_t j = 0; j < k; ++j) {
                double term = (double)vals[bi[j] * 3 + c] * w[j];
                acc = j == 0 ? term : acc + term;
            }
            out[q * 3 + c] = (float)acc;
        }
        if (nbr_out)
            for (int64_t j = 0; j < k; ++j) nbr_out[q * k + j] = bi[j];
    }
}

/* ---- chamfer_distance_chunked_optimized row minima (losses.py:24-59) ----------------------
 * D = (|p|^2 + |q|^2) + (-2 * dot), clamp >= 0, min over q; returns min and argmin (first
 * index on ties).  One direction; call twice with swapped roles. */
void orc_chamfer_rowmin(const float* P, int64_t N, const float* Qp, int64_t M, float* mind,
                        int64_t* argmin) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < N; ++i) {
        const float* p = P + i * 3;
        float np_ = sqnorm3(p);
        float best = INFINITY;
        int64_t bj = 0;
        for (int64_t j = 0; j < M; ++j) {
            const float* q = Qp + j * 3;
            float d = (np_ + sqnorm3(q)) + (-2.0f * dot3_fma(p, q));
            if (d < 0.0f) d = 0.0f;
            if (d < best) { best = d; bj = j; }
        }
        mind[i] = best;
        argmin[i] = bj;
    }
}
