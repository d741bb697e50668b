/*
 * oracle/labcu_restate.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Lane-level CPU restatement of the reference's `order_array` pipeline
 * (`Sord Radix y Merge/lab.cu`, referred to below as lab.cu).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this file's
 * library; the product (liblabsort.so) never links or calls it.
 *
 * Why it exists: the reference has no tests and no golden outputs,
 * and lab.cu cannot be built here (CUDA only: no nvcc, and a HIP build would
 * need stand-in CUDA headers, which this task forbids).  This restatement is
 * what lab.cu computes, step by step, so the test-suite can (a) show where the
 * reference's own result equals std::sort (the spec, letra.pdf p.3 "Consigna")
 * and (b) document the reference's failure modes:
 *   F4  launch failure for n >= 2^18 (block > 1024 threads) or when the
 *       separators kernel needs > 48 KiB of dynamic shared memory  -> LABCU_LAUNCH_FAIL
 *   F5  off-by-one co-rank at lab.cu:253-260 (inclusive end passed as a size)
 *       -> mis-ordered output; segments > 512 keys -> out-of-bounds shared
 *       accesses / dropped keys                                       -> LABCU_UB
 *   F6  negative keys make radix_sort_kernel spin forever               -> LABCU_HANG
 *
 * Execution model emulated:
 *   - blocks run one after another, threads of a block run phase by phase
 *     (one phase = code between two __syncthreads / __syncwarp);
 *   - __shfl_up/down_sync return the lane's own value when the source lane is
 *     out of range; __all_sync is an AND over the 32 lanes;
 *   - int32 arithmetic wraps (lane 0's "previous" value is cur-1, lab.cu:57-58).
 * `fix_f5` makes the search end at lab.cu:254 exclusive, which is the one-line
 * change that makes the pipeline correct for every tested input up to 2^17.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define LABCU_OK 0
#define LABCU_LAUNCH_FAIL 1
#define LABCU_HANG 2
#define LABCU_UB 3
#define LABCU_BAD_ARG 4

#define WARP 32

/* ---- lab.cu:11-41  exlusiveScan: Blelloch up/down sweep through shuffles ---- */
static void warp_exclusive_scan(int v[WARP]) {
    int offset = 1;
    /* up-sweep, lab.cu:17-22 */
    while (offset < WARP) {
        int pre[WARP];
        for (int l = 0; l < WARP; ++l) pre[l] = (l - offset >= 0) ? v[l - offset] : v[l];
        for (int l = 0; l < WARP; ++l)
            if (((l + 1) % (offset * 2)) == 0) v[l] += pre[l];
        offset *= 2;
    }
    v[WARP - 1] = 0; /* lab.cu:24-26 */
    /* down-sweep, lab.cu:29-39 */
    offset /= 2;
    while (offset > 0) {
        int sup[WARP], inf[WARP];
        for (int l = 0; l < WARP; ++l) {
            sup[l] = (l + offset < WARP) ? v[l + offset] : v[l];
            inf[l] = (l - offset >= 0) ? v[l - offset] : v[l];
        }
        for (int l = 0; l < WARP; ++l) {
            int dbl = ((l + 1) % (offset * 2)) == 0;
            v[l] += dbl ? inf[l] : 0;
            v[l] = (!dbl && ((l + 1) % offset) == 0) ? sup[l] : v[l];
        }
        offset /= 2;
    }
}

static int wrap_dec(int x) { return (int)((uint32_t)x - 1u); }

static int warp_all_sorted(const int cur[WARP]) {
    /* lab.cu:56-58 and :80-83: prev = shfl_up(cur,1); lane 0's prev = cur-1 */
    for (int l = 0; l < WARP; ++l) {
        int prev = (l == 0) ? wrap_dec(cur[0]) : cur[l - 1];
        if (!(prev <= cur[l])) return 0;
    }
    return 1;
}

/* ---- lab.cu:47-87  radix_sort_kernel on one 32-key tile ---- */
static int radix_tile(int *src) {
    int cur[WARP];
    memcpy(cur, src, sizeof(cur));
    uint32_t mask = 1; /* `int mask` shifted left: 1<<31 then 0 (lab.cu:60,78) */
    while (!warp_all_sorted(cur)) {
        if (mask == 0) return LABCU_HANG; /* every further iteration is the identity (F6) */
        int flag[WARP], scan[WARP];
        for (int l = 0; l < WARP; ++l) flag[l] = (((uint32_t)cur[l] & mask) == 0) ? 1 : 0;
        memcpy(scan, flag, sizeof(scan));
        warp_exclusive_scan(scan);
        int total_false = flag[WARP - 1] + scan[WARP - 1]; /* lab.cu:66-67 */
        int swap[WARP];
        for (int l = 0; l < WARP; ++l) {
            int t = l - scan[l] + total_false;           /* lab.cu:69 */
            int np = flag[l] ? scan[l] : t;              /* lab.cu:70 */
            swap[np] = cur[l];                           /* lab.cu:72 (tie = 0) */
        }
        memcpy(cur, swap, sizeof(cur));                 /* lab.cu:76 */
        mask <<= 1;
    }
    memcpy(src, cur, sizeof(cur));
    return LABCU_OK;
}

/* ---- lab.cu:102-132  busquedaPorBiparticion ---- */
static int bsearch_ref(const int *arr, int start, int size, int x, int before_equal) {
    if (size <= 0) return 0;
    int fin = start + size - 1, ini = start, mid = (ini + fin) / 2;
    while (ini < fin) {
        int pivot = arr[mid];
        int down = before_equal ? (x <= pivot) : (x < pivot);
        ini = down ? ini : mid + 1;
        fin = down ? mid : fin;
        mid = (ini + fin) / 2;
    }
    int pivot = arr[mid];
    if (before_equal) return (pivot < x ? mid + 1 : mid) - start;
    return (pivot > x ? mid : mid + 1) - start;
}

/* Shared-memory view with bounds tracking: accesses outside the declared
 * shared array are undefined behaviour in the reference; we flag them. */
typedef struct {
    int *a;
    int cap;
    int ub;
} shmem_t;

static int sh_get(shmem_t *s, int i) {
    if (i < 0 || i >= s->cap) { s->ub = 1; return 0; }
    return s->a[i];
}
static void sh_set(shmem_t *s, int i, int v) {
    if (i < 0 || i >= s->cap) { s->ub = 1; return; }
    s->a[i] = v;
}

/* binary search that reads through the bounds-checked shared array */
static int bsearch_sh(shmem_t *s, int start, int size, int x, int before_equal) {
    if (size <= 0) return 0;
    int fin = start + size - 1, ini = start, mid = (ini + fin) / 2;
    while (ini < fin) {
        int pivot = sh_get(s, mid);
        int down = before_equal ? (x <= pivot) : (x < pivot);
        ini = down ? ini : mid + 1;
        fin = down ? mid : fin;
        mid = (ini + fin) / 2;
    }
    int pivot = sh_get(s, mid);
    if (before_equal) return (pivot < x ? mid + 1 : mid) - start;
    return (pivot > x ? mid : mid + 1) - start;
}

/* ---- lab.cu:144-182  deviceOrderedJoin for one block of `bdim` threads ---- */
static void ordered_join(const int *src, int posA, int lenA, int posB, int lenB, int *out, int posOut,
                         shmem_t *sh, int bdim, int n_global, int *ub) {
    int active = lenA + lenB;
    if (active > bdim) { active = bdim; *ub = 1; } /* keys past blockDim are silently dropped */
    int *val = (int *)malloc(sizeof(int) * (size_t)(active > 0 ? active : 1));
    int *isb = (int *)malloc(sizeof(int) * (size_t)(active > 0 ? active : 1));
    int *idm = (int *)malloc(sizeof(int) * (size_t)(active > 0 ? active : 1));
    int *rk = (int *)malloc(sizeof(int) * (size_t)(active > 0 ? active : 1));
    for (int t = 0; t < active; ++t) { /* lab.cu:153-158 */
        isb[t] = t >= lenA;
        idm[t] = isb[t] ? t - lenA : t;
        int g = isb[t] ? posB + idm[t] : posA + idm[t];
        if (g < 0 || g >= n_global) { *ub = 1; val[t] = 0; } else val[t] = src[g];
        sh_set(sh, t, val[t]);
    }
    for (int t = 0; t < active; ++t) /* lab.cu:170 */
        rk[t] = bsearch_sh(sh, isb[t] ? 0 : lenA, isb[t] ? lenA : lenB, val[t], !isb[t]);
    for (int t = 0; t < active; ++t) sh_set(sh, idm[t] + rk[t], val[t]); /* lab.cu:175 */
    for (int t = 0; t < active; ++t) {                                  /* lab.cu:180 */
        int g = posOut + t;
        if (g < 0 || g >= n_global) { *ub = 1; continue; }
        out[g] = sh_get(sh, t);
    }
    if (sh->ub) *ub = 1;
    free(val); free(isb); free(idm); free(rk);
}

/*
 * labcu_order_array: restatement of lab.cu:303-402 on a host array.
 *   data   in/out, n keys (the reference requires a power of two, 32 <= n)
 *   fix_f5 0 = as written; 1 = exclusive search end at lab.cu:254
 * Returns LABCU_* status; data holds what the reference would copy back
 * (meaningful only for LABCU_OK / LABCU_UB).
 */
int labcu_order_array(int *data, int n, int fix_f5) {
    if (n < 32 || (n & (n - 1)) != 0) return LABCU_BAD_ARG;
    int ub = 0;
    /* stage 1: radix_sort_kernel<<<n/32, 32>>> (lab.cu:325-330) */
    for (int b = 0; b < n / 32; ++b) {
        int st = radix_tile(data + (size_t)b * 32);
        if (st != LABCU_OK) return st;
    }
    /* stage 2: orderedJoin, block sizes 64..min(512,n) (lab.cu:334-346) */
    int bs = 64;
    int lim = n < 512 ? n : 512;
    while (bs <= lim) {
        int *sharr = (int *)malloc(sizeof(int) * (size_t)bs);
        for (int b = 0; b < n / bs; ++b) {
            shmem_t sh = {sharr, bs, 0};
            int base = b * bs;
            ordered_join(data, base, bs / 2, base + bs / 2, bs / 2, data, base, &sh, bs, n, &ub);
        }
        free(sharr);
        bs *= 2;
    }
    bs /= 2;
    if (bs >= n) return ub ? LABCU_UB : LABCU_OK;

    /* stage 3 (lab.cu:350-391) */
    int *src = data;
    int *dst = (int *)malloc(sizeof(int) * (size_t)n);
    for (int i = 0; i < n; ++i) dst[i] = (int)0x7EADBEEF; /* cudaMalloc content: unknown */
    int sep_len = n / 32;                                /* lab.cu:311 */
    int *sep_a = (int *)calloc((size_t)sep_len, sizeof(int)); /* memset 0, lab.cu:318-319 */
    int *sep_b = (int *)calloc((size_t)sep_len, sizeof(int));
    int sector = bs;
    int t = bs / 2;
    int status = LABCU_OK;
    while (sector < n) {
        sector *= 2;
        int qty = (n + sector - 1) / sector;
        int sps = 2 * (1 + ((sector / 2) + t - 1) / t);
        size_t shmem = (size_t)sps * (size_t)qty * sizeof(int) * 2; /* lab.cu:372 */
        if (sps > 1024 || shmem > 48 * 1024) { status = LABCU_LAUNCH_FAIL; break; }
        int half = sps / 2;
        /* separators_kernel, lab.cu:209-270, one block per sector */
        int *sv = (int *)malloc(sizeof(int) * (size_t)sps);
        int *sg = (int *)malloc(sizeof(int) * (size_t)sps);
        for (int sid = 0; sid < qty; ++sid) {
            for (int k = 0; k < sps; ++k) { /* phase 1: lab.cu:217-232 */
                int is_a = k < half;
                int lim2 = sid * sector + (is_a ? sector / 2 : sector);
                if (lim2 > n) lim2 = n;
                int pos = sid * sector + (k % half) * t + (is_a ? 0 : sector / 2);
                if (pos >= lim2) pos = lim2 - 1;
                sv[k] = src[pos];
                sg[k] = pos;
            }
            for (int k = 0; k < sps; ++k) { /* phase 2: lab.cu:240-269 */
                int is_a = k < half;
                int value = sv[k];
                int pos = sg[k];
                int s_off = is_a ? half : 0;
                int s_opp = bsearch_ref(sv, s_off, half, value, is_a);
                int s_start, s_end;
                if (s_opp <= 0) s_start = sid * sector + (is_a ? sector / 2 : 0);
                else s_start = sg[s_opp + s_off - 1];
                if (s_opp >= half - 1) {
                    int e = sid * sector + (is_a ? sector : sector / 2);
                    if (!fix_f5) { e -= 1; if (e > n - 1) e = n - 1; } /* lab.cu:254 as written */
                    else if (e > n) e = n;                            /* exclusive end (fix) */
                    s_end = e;
                } else {
                    s_end = sg[s_opp + s_off + 1];
                }
                int opp = bsearch_ref(src, s_start, s_end - s_start, value, is_a) + s_start;
                int pa = is_a ? pos : opp;
                int pb = is_a ? opp : pos;
                int sp = is_a ? (k + s_opp) : (k % half + s_opp);
                int o = sid * sps + sp;
                if (o < 0 || o >= sep_len) { ub = 1; continue; }
                sep_a[o] = pa;
                sep_b[o] = pb;
            }
        }
        free(sv);
        free(sg);
        /* merge_segments_kernel<<<(sps, qty), 512>>>, lab.cu:272-300 */
        int sharr[512];
        for (int sid = 0; sid < qty; ++sid) {
            for (int seg = 0; seg < sps; ++seg) {
                int sp = sid * sps + seg;
                int sa = sep_a[sp], sb = sep_b[sp];
                int off = sid * sector;
                int ea, eb;
                if (seg == sps - 1) { ea = off + sector / 2; eb = off + sector; }
                else { ea = sep_a[sp + 1]; eb = sep_b[sp + 1]; }
                int dpos = sa + sb - off - sector / 2;
                shmem_t sh = {sharr, 512, 0};
                int la = ea - sa; if (la < 0) la = 0;
                int lb = eb - sb; if (lb < 0) lb = 0;
                ordered_join(src, sa, la, sb, lb, dst, dpos, &sh, 512, n, &ub);
            }
        }
        int *aux = src; src = dst; dst = aux;
    }
    if (status == LABCU_OK && src != data) memcpy(data, src, sizeof(int) * (size_t)n);
    if (src != data) free(src); else free(dst);
    free(sep_a);
    free(sep_b);
    if (status != LABCU_OK) return status;
    return ub ? LABCU_UB : LABCU_OK;
}

/* Stage-1 only (lab.cu:47-87 over n/32 tiles): exposes the tile radix so the
 * per-tile behaviour (early exit, F6 hang) can be tested in isolation. */
int labcu_radix_tiles(int *data, int n) {
    if (n < 0 || n % 32) return LABCU_BAD_ARG;
    for (int b = 0; b < n / 32; ++b) {
        int st = radix_tile(data + (size_t)b * 32);
        if (st != LABCU_OK) return st;
    }
    return LABCU_OK;
}

/* Exposes lab.cu:11-41 for the unit tests (32 ints in, exclusive scan out). */
void labcu_warp_scan(int *v32) { warp_exclusive_scan(v32); }

/* Exposes lab.cu:102-132 for the unit tests. */
int labcu_bsearch(const int *arr, int start, int size, int x, int before_equal) {
    return bsearch_ref(arr, start, size, x, before_equal);
}
