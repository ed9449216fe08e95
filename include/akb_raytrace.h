/*
 * akb_raytrace.h — C ABI of the MI355X-native AKB ray-trace / wavefront / PSF hot path.
 *
 * One shared library, akbraytracing_amd/lib/libakb_hip.so, built by hipcc for gfx950.
 * Every entry point:
 *   - takes plain pointers and sizes (no torch / numpy types),
 *   - treats every array pointer as DEVICE memory unless the name says host,
 *   - is stream-ordered on the hipStream_t passed as `void* stream` (NULL = default stream),
 *   - returns 0 on success or a negative AKB_E* code; akb_last_error() gives the message
 *     (thread-local, valid until the next call on the same thread). No C++ exception crosses it.
 *
 * Arrays of 3-vectors use the reference's struct-of-arrays layout: a (3, N) float64 C-order
 * block, row k (x/y/z) at base + k*ld, element i at + i*inc. inc = 0 broadcasts one vector
 * (the reference's `ray` of shape (3,)). ld = N, inc = 1 is the plain numpy (3, N) array.
 *
 * Reference interface each entry point replaces (file:line under Kakekakechan/AKBRaytracing):
 *   akb_isect_f64        mirr_ray_intersection   EllipseRaytrace3D.py:18-45, AKB_raytrace_20250312.py:444-471
 *   akb_normal_f64       norm_vector             EllipseRaytrace3D.py:61-71, AKB_raytrace_20250312.py:626-636
 *   akb_reflect_f64      reflect_ray             EllipseRaytrace3D.py:47-55, AKB_raytrace_20250312.py:501-509
 *   akb_normalize_f64    normalize_vector        EllipseRaytrace3D.py:57-59, AKB_raytrace_20250312.py:530-532
 *   akb_plane_isect_f64  plane_ray_intersection  EllipseRaytrace3D.py:145-157, AKB_raytrace_20250312.py:873-885
 *   akb_seglen_f64       np.linalg.norm(b-a, axis=0)  AKB_raytrace_20250312.py:2884-2897, :3623, :3630
 *   akb_rotate_f64       rotate_vectors / rotate_points  AKB_raytrace_20250312.py:917-943
 *   akb_trace_chain_f64  the pass-1 / pass-2 mirror chains of plot_result_debug
 *                        AKB_raytrace_20250312.py:2694-2717 (ray grid), :2770-2845 (pass 1),
 *                        :2881-2905 (pass 2 + OPL segments); KB_debug :10952-10997
 *   akb_tilt_opd_f64     tilt correction + detector + OPL/OPD, AKB_raytrace_20250312.py:3583-3601, :3611-3677
 *   akb_pairwise_sum_f64 np.sum / np.mean / np.nanmean as used at :3583-3591, :3626, :3633, :3674
 *   akb_huygens_f64      compute_u_parallel / forward_propagation_*_batch
 *                        Wavecalc_raytrace_fromData_CPU0402.py:71-124, ..._GPU0402.py:64-201
 *   akb_psf_f64          compute_psf_fft         psf_fft.py:29-125 (FFT on rocFFT)
 *   akb_trace_chain_batch_f64 + akb_focus_eval_f64
 *                        plot_result_debug(params, 'test') / auto_focus_NA's sweeps
 *                        AKB_raytrace_20250312.py:2770-2847, :3565-3601, :12746-12895
 *   akb_sep_search_f64   compare_sep / optimize_min_index of plot_result_debug(params, 'sep') and
 *                        auto_focus_sep, AKB_raytrace_20250312.py:9174-9560, :3604-3606, :12897-13318
 */
#ifndef AKB_RAYTRACE_H
#define AKB_RAYTRACE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AKB_ABI_VERSION 17

/* status codes */
#define AKB_OK 0
#define AKB_E_INVALID (-1)   /* bad argument (shape, pointer, size) */
#define AKB_E_HIP (-2)       /* HIP runtime error */
#define AKB_E_FFT (-3)       /* rocFFT error */
#define AKB_E_NOMEM (-4)     /* allocation failed */

/* bits of the device int32 `flags` word written by the trace kernels */
#define AKB_FLAG_MISS 0x1          /* some ray had discriminant D <= 0 (or NaN): ref :457 all-NaN rule */
#define AKB_FLAG_ZERO_NORMAL 0x2   /* some surface normal had zero norm: ref :530-532 passthrough rule */
#define AKB_FLAG_ZERO_REFLECT 0x4  /* some reflected direction had zero norm */
#define AKB_FLAG_ZERO_DIR 0x8      /* some generated initial direction had zero norm */
/* akb_trace_chain_f64 shifts the MISS/ZERO bits of mirror k by 4*k (k < 7); bit 28
 * (AKB_FLAG_CHAIN_DIR) marks a zero-norm generated initial direction */
#define AKB_FLAG_CHAIN_DIR (1 << 28)

const char* akb_last_error(void);
int akb_abi_version(void);
/* sha256 (hex) of the sources this library was compiled from: every csrc/ file the build compiles
 * or includes plus this header, as akbraytracing_amd/build.py:sources_hash() forms it. The Python
 * binding refuses a library whose hash differs from the tree's (a stale prebuilt .so). */
const char* akb_sources_hash(void);
/* number of visible HIP devices (0 on a host without GPU; never fails) */
int akb_device_count(void);
/* a stream on the current device whose kernels leave `reserve` CUs (a multiple of 8 up to 128;
 * the same number on every XCD) to the device's other streams: the trace's passes run on it so that the
 * faithful chain's single-workgroup kernels find a free CU at once instead of waiting for one to
 * drain of pass workgroups. *stream receives the hipStream_t; release it with akb_stream_destroy
 * (a stream still alive when the library unloads is destroyed then). */
int akb_stream_create_reserved(int reserve, void** stream);
/* the CU mask such a stream gets on a device of ncu CUs (ncu / 32 words; host only, no device call) */
int akb_reserved_cu_mask(int reserve, int ncu, uint32_t* mask);
int akb_stream_destroy(void* stream);

/* ---------------- stage primitives (drop-in boundary, one reference call each) ---------------- */

/* mirr_ray_intersection: point = t*dir + org, t = (-B +- sqrt(B^2-4AC)) / (2A), minus root when
 * negative != 0. Writes `out` for every ray and ORs AKB_FLAG_MISS into *flags if any D <= 0;
 * the caller then replaces the whole output by NaN (reference :457-459). */
int akb_isect_f64(const double coeffs[10], const double* dir, int64_t dir_ld, int64_t dir_inc,
                  const double* org, int64_t org_ld, int64_t org_inc, int negative, int64_t n,
                  double* out, int64_t out_ld, int32_t* flags, void* stream);

/* norm_vector: gradient of the quadric at `pt`, normalised. normalize=1 writes the unit normal
 * and ORs AKB_FLAG_ZERO_NORMAL if any norm == 0; normalize=0 writes the raw gradient (the
 * reference's passthrough when any norm is zero). */
int akb_normal_f64(const double coeffs[10], const double* pt, int64_t pt_ld, int64_t pt_inc, int64_t n,
                   double* out, int64_t out_ld, int normalize, int32_t* flags, void* stream);

/* reflect_ray: phai = dir - 2 (dir.N) N, normalised as akb_normal_f64 (AKB_FLAG_ZERO_REFLECT). */
int akb_reflect_f64(const double* dir, int64_t dir_ld, int64_t dir_inc, const double* nrm,
                    int64_t nrm_ld, int64_t nrm_inc, int64_t n, double* out, int64_t out_ld,
                    int normalize, int32_t* flags, void* stream);

/* normalize_vector: out = v / ||v|| ; ORs AKB_FLAG_ZERO_DIR if any ||v|| == 0 (caller keeps v). */
int akb_normalize_f64(const double* v, int64_t v_ld, int64_t v_inc, int64_t n, double* out,
                      int64_t out_ld, int32_t* flags, void* stream);

/* plane_ray_intersection with plane g x + h y + i z + j = 0 (coeffs[6:10]); per-ray inf/NaN. */
int akb_plane_isect_f64(const double ghij[4], const double* dir, int64_t dir_ld, int64_t dir_inc,
                        const double* org, int64_t org_ld, int64_t org_inc, int64_t n, double* out,
                        int64_t out_ld, void* stream);

/* out[i] = sqrt(((bx-ax)^2 + (by-ay)^2) + (bz-az)^2) */
int akb_seglen_f64(const double* a, int64_t a_ld, int64_t a_inc, const double* b, int64_t b_ld,
                   int64_t b_inc, int64_t n, double* out, void* stream);

/* out = Ry @ (Rz @ (v - c)) + c with c = center (host 3-vector, or NULL for rotate_vectors).
 * ry, rz: host row-major 3x3 matrices. Each product row is fma(r2, v2, fma(r1, v1, r0*v0)),
 * the order OpenBLAS dgemm uses for the reference's matmul. */
int akb_rotate_f64(const double ry[9], const double rz[9], const double center[3], const double* v,
                   int64_t v_ld, int64_t v_inc, int64_t n, double* out, int64_t out_ld, void* stream);

/* fill rows x n of `out` (row stride ld) with quiet NaN */
int akb_fill_nan_f64(double* out, int64_t ld, int rows, int64_t n, void* stream);

/* ---------------- numpy-order reductions fused into producer kernels ---------------- */

/* A producer kernel that owns a leaf sink reduces up to 8 per-ray quantities on the fly, in
 * numpy's summation order: for every full 8192-element buffer it writes the 64 pairwise leaf
 * sums (128 consecutive elements, 8 accumulators each) and their non-NaN counts, and it copies
 * the raw values of the short last buffer; akb_leaf_finish_f64 then completes np.sum /
 * np.nanmean exactly as akb_pairwise_sum_f64 would on the materialised rows, without those rows
 * ever reaching HBM. Lay one out with akb_leaf_sink_layout over akb_leaf_sink_bytes of memory. */
typedef struct akb_leaf_sink {
    double* leaf_sum;   /* [nq][n_full_leaves] */
    int32_t* leaf_cnt;  /* [nq][n_full_leaves] */
    double* tail;       /* [nq][8192] */
    int32_t nq;         /* 0 disables the sink */
    int32_t nan_mask;   /* bit q set: NaN -> 0 and not counted (np.nansum / np.nanmean); q >= 31 use bit 31 */
    int64_t n;          /* elements reduced per quantity */
} akb_leaf_sink;

int64_t akb_leaf_sink_bytes(int nq, int64_t n);
int akb_leaf_sink_layout(void* base, int nq, int nan_mask, int64_t n, akb_leaf_sink* out);
int64_t akb_leaf_finish_work_bytes(int nq, int64_t n);
/* d_sum[nq], d_count[nq] (device) */
int akb_leaf_finish_f64(const akb_leaf_sink* sink, double* d_sum, int64_t* d_count, void* work,
                        void* stream);
/* The two halves of akb_leaf_finish_f64, for a sum spread over ranks whose shards are aligned to
 * numpy's 8192-element buffers (every shard but the last a whole number of buffers): each rank
 * forms its full buffers' sums d_part[q * part_ld + c] and counts, and its short last buffer's
 * pairwise sum and count (zero when its shard has none; only the last rank's can be non-empty)... */
int akb_leaf_parts_f64(const akb_leaf_sink* sink, double* d_part, int64_t* d_part_cnt, int part_ld,
                       double* d_tail_sum, int64_t* d_tail_cnt, void* stream);
/* ... and, with every rank's buffer sums gathered in grid order (q-major rows of part_ld), adds
 * them left to right as numpy does: d_sum[q], d_count[q]. The caller adds the last rank's short
 * buffer sum last (sum = chain + tail), which is numpy's order exactly: the cross-rank result
 * equals the single-process one bit for bit. */
int akb_parts_chain_f64(const double* d_part, const int64_t* d_part_cnt, int part_ld, int nq, int nparts,
                        double* d_sum, int64_t* d_count, void* stream);

/* ---------------- fused chain (device-resident API) ---------------- */

#define AKB_MAX_MIRRORS 7

typedef struct akb_chain_desc {
    int32_t n_mirrors;                       /* K <= AKB_MAX_MIRRORS */
    int32_t negative[AKB_MAX_MIRRORS];       /* minus root per mirror (ref :2820 H-hyperboloid) */
    double coeffs[AKB_MAX_MIRRORS][10];      /* quadric a..j per mirror, in trace order */
    double det_ghij[4];                      /* detector plane for det_out */
    /* initial rays: either explicit (dir != NULL) or generated on the grid
     * dir[:, iv*n_h + ih] = normalize(1, tan_h[ih], tan_v[iv])   (ref :2711-2717) */
    const double* dir; int64_t dir_ld; int64_t dir_inc;
    const double* tan_h; const double* tan_v; int64_t n_h; int64_t n_v;
    int64_t ray0;                            /* first flat ray index iv*n_h + ih of this launch (a
                                              * multi-GPU shard; RayWave aligns shards to numpy's
                                              * 8192-element sum buffers) */
    int64_t n_rays;                          /* rays in this launch */
    const double* org; int64_t org_ld; int64_t org_inc; /* NULL => constant source src[] */
    double src[3];
    /* outputs (any may be NULL) */
    double* hits; int64_t hits_ld;           /* K blocks of (3, hits_ld): mirror hit points */
    double* last_hit; int64_t last_hit_ld;   /* (3, ld) point on the last mirror */
    double* dir_out; int64_t dir_out_ld;     /* (3, ld) direction after the last mirror */
    double* det_out; int64_t det_out_ld;     /* (3, ld) hit on det_ghij */
    double* opl;                             /* (n): ((d01 + d12) + d23) + ... left to right */
    double* atan_h; double* atan_v;          /* (n): arctan(Ry/Rx), arctan(Rz/Rx) of dir_out */
    /* exit-slope samples for the equal-angle resample (ref :2849-2870); the caller applies
     * np.arctan on the host so the resampled tables stay bit-identical to the reference */
    int64_t samp_h_begin; int64_t samp_h_end; /* flat ray range -> samp_h[i - begin] = Ry/Rx */
    int64_t samp_v_col;                       /* column ih -> samp_v[iv] = Rz/Rx */
    double* samp_h; double* samp_v;
    int32_t* flags;                           /* device int32, OR-ed */
    /* optional fused reduction of (atan_h, atan_v, det_x, det_y, det_z): sink.nq = 5 */
    akb_leaf_sink sink;
    /* optional per-ray OPL perturbation on the grid (BASELINE config 5, a figure-error model on a
     * Legendre basis; grid rays only, needs opl): opl += sum_t pert_v[t][iv] * pert_h[t][ih] for
     * t < pert_terms (<= 8), tables (pert_terms, n_v) and (pert_terms, n_h), row-major */
    const double* pert_h; const double* pert_v; int32_t pert_terms;
    /* optional staging copy done by the launch itself (not part of the trace): copy_n doubles from
     * copy_src (e.g. pinned host memory the caller filled before the launch) to copy_dst (device
     * memory a later launch on the stream reads) - RayWave hands the next pass 2 its resampled
     * tables this way, with no copy packet between the two trace kernels */
    const double* copy_src; double* copy_dst; int64_t copy_n;
} akb_chain_desc;

int akb_trace_chain_f64(const akb_chain_desc* desc, void* stream);
/* sizeof(akb_chain_desc), for bindings to check their struct layout */
int64_t akb_chain_desc_size(void);

/* tilt + detectors + OPL (ref :3583-3601, :3611-3633):
 *   r' = Ry@(Rz@r), p' = Ry@(Rz@(p - c)) + c
 *   det1 = plane(det1_ghij, r', p'), det2 = plane(det2_ghij, r', p')
 *   total1 = opl + ||det1 - p'||, total2 = opl + ||det2 - p'||
 * Any output may be NULL. sink (optional, nq = 5): fused np.nanmean of
 * (det1_x, det1_y, det1_z, total1, total2). */
int akb_tilt_opd_f64(const double ry[9], const double rz[9], const double center[3],
                     const double det1_ghij[4], const double det2_ghij[4], const double* dir,
                     const double* pt, const double* opl, int64_t ld, int64_t n, double* dir_rot,
                     double* pt_rot, double* det1, double* det2, double* total1, double* total2,
                     const akb_leaf_sink* sink, void* stream);

/* The tilt parameters on the device (ref :3583-3591, rotate_vectors :917-927), so nothing waits
 * on the host between pass 2 and the tilt. From the pass-2 sink's sums / counts of (arctan(Ry/Rx),
 * arctan(Rz/Rx), det_x, det_y, det_z) it writes d_params[23]:
 *   [0] theta_y = -nanmean(arctan(Rz/Rx))   [1] theta_z = nanmean(arctan(Ry/Rx))
 *   [2..10] R_y, [11..19] R_z (row-major) of rotation_matrices(-theta_y, -theta_z), formed with
 *           correctly rounded cos / sin (glibc's differ from those on ~0.13 % of arguments)
 *   [20..22] focus_apprx = mean(det) (np.mean)
 *   [23..24] the first four int32 words of d_clear as they were (zero-padded)
 * and zeroes d_extent_keys[4] (optional) and d_clear[0..n_clear) (e.g. the trace flag words, read
 * back from [23..24]) for the next step. d_params holds 25 doubles. */
int akb_tilt_params_f64(const double* d_sum5, const int64_t* d_cnt5, double* d_params, uint64_t* d_extent_keys,
                        int32_t* d_clear, int n_clear, void* stream);

/* akb_leaf_finish_f64 + akb_tilt_params_f64 for the pass-2 sink in two small launches instead of
 * three (nq = 5: arctan(Ry/Rx), arctan(Rz/Rx), det x, y, z; one process, sums over the whole sink):
 * d_sum5 / d_cnt5 and the parameter block exactly as the two calls give them.
 * work: akb_finish_params_work_bytes(sink). */
int64_t akb_finish_params_work_bytes(const akb_leaf_sink* sink);
int akb_finish_tilt_params_f64(const akb_leaf_sink* sink, double* d_sum5, int64_t* d_cnt5, double* d_params,
                               uint64_t* d_extent_keys, int32_t* d_clear, int n_clear, void* work, void* stream);

/* akb_tilt_opd_f64 with R_y, R_z and the centre read from akb_tilt_params_f64's device block. */
int akb_tilt_opd_dev_f64(const double* d_params, const double det1_ghij[4], const double det2_ghij[4],
                         const double* dir, const double* pt, const double* opl, int64_t ld, int64_t n,
                         double* dir_rot, double* pt_rot, double* det1, double* det2, double* total1,
                         double* total2, const akb_leaf_sink* sink, void* stream);

/* The resample picks of a pass-1 descriptor alone: traces only the rays whose exit slopes the
 * equal-angle resample reads (the middle-row range samp_h_begin..samp_h_end and grid column
 * samp_v_col, ref AKB_raytrace_20250312.py:2849-2859) over the whole grid (ray0 / n_rays ignored),
 * writing samp_h / samp_v and ORing their flags. RayWave runs it ahead of the full pass 1 so the
 * host resample overlaps the full trace (whose flags it checks after pass 2). */
int akb_trace_chain_samples_f64(const akb_chain_desc* d, void* stream);

/* Pass 1 of one run fused with the device-parameter tilt of the previous run (RayWave's pipelined
 * mode): one launch traces the chain descriptor d (grid rays, no OPL, no sink: pass 1, ref
 * AKB_raytrace_20250312.py:2805-2838) and applies akb_tilt_opd_dev_f64's tilt to the n rays of
 * dir / pt / opl (the previous run's pass-2 outputs, ref :3583-3633) over the same shard. The
 * tilt's loads overlap the chain's FP64 arithmetic inside each wave. Outputs and flags are those
 * of the two calls; d->n_rays must equal n. */
int akb_chain_tilt_f64(const akb_chain_desc* d, const double* d_params, const double det1_ghij[4],
                       const double det2_ghij[4], const double* dir, const double* pt, const double* opl, int64_t ld,
                       int64_t n, double* dir_rot, double* pt_rot, double* det1, double* det2, double* total1,
                       double* total2, const akb_leaf_sink* sink, void* stream);
/* akb_chain_tilt_f64 (detector-2 rows) that also forms the OPD maps of the run before the tilted
 * one (akb_opd_f64 without detector 1 / Sph): from that run's opd_total2 (n) and opd_det2 (3, ld)
 * and its tilt sums d_sum5 / d_cnt5, dist_err2 = (total2 - mean2) * 1e9, wave = dist_err2 - Sph,
 * and its detector-2 extents max-folded into d_extent_keys (zeroed beforehand, e.g. by
 * akb_tilt_params_f64). Same n and ld as the tilt. The chain's resample picks, the tilt and the
 * OPD are those of the three separate calls. */
int akb_chain_tilt_opd_f64(const akb_chain_desc* d, const double* d_params, const double det1_ghij[4],
                           const double det2_ghij[4], const double* dir, const double* pt, const double* opl,
                           int64_t ld, int64_t n, double* det2, double* total2, const akb_leaf_sink* sink,
                           const double* opd_total2, const double* opd_det2, const double* d_sum5,
                           const int64_t* d_cnt5, double* dist_err2, double* wave, uint64_t* d_extent_keys,
                           void* stream);

/* S independent systems in one launch (auto_focus_NA / calc_FoC trace many small systems, ref
 * AKB_raytrace_20250312.py:12776-12786, :13780-13784): descs[s] is an akb_trace_chain_f64 descriptor
 * (host array) with grid rays, no sink, resample picks or staging copy, and every system asking for
 * the same opl / hits rows. Each system's outputs and flag word are its own. */
int akb_trace_chain_batch_f64(const akb_chain_desc* descs, int n_sys, void* stream);

/* The focus evaluation of plot_result_debug's 'test' mode and auto_focus_NA's spot sizes (ref
 * :2842-2847, :3565-3601, :12785-12786) for traced rays: system s has its exit directions and last
 * hits at dir / pt + s * sys_ld ((3, n) rows each) and n_planes detector planes x = -j,
 * d_plane_j[s * n_planes + p] (coeffs_det[9]). d_rot (device, (n_sys, 18): R_y then R_z of
 * rotate_vectors, row-major) applies the tilt - det0 = plane(dir, pt), focus = np.mean(det0, axis=1),
 * dir' = R_y@(R_z@dir), pt' = R_y@(R_z@(pt - focus)) + focus, det = plane(dir', pt') - or NULL for
 * option_tilt=False (det = det0). d_std (n_sys * n_planes, 2) = np.std(det[2]), np.std(det[1]), every
 * sum in numpy's order. det_out / dir_out (optional, (n_sys * n_planes, 3, n)): det and the
 * (tilted) directions, the 'test' return's detcenter and angle. work: akb_focus_eval_work_bytes. */
int64_t akb_focus_eval_work_bytes(int n_sys, int n_planes, int64_t n);
int akb_focus_eval_f64(const double* dir, const double* pt, int64_t n, int64_t sys_ld, int n_sys, int n_planes,
                       const double* d_plane_j, const double* d_rot, double* d_std, double* det_out, double* dir_out,
                       void* work, void* stream);

/* compare_sep's plane searches (ref AKB_raytrace_20250312.py:9267-9560; optimize_min_index :9174-9217,
 * create_func_to_minimize / create_evaluation_fn :9219-9265), all in one launch. Search q minimises
 * sqrt(np.std(z)^2 + np.std(y)^2) of the hits of rays start[q] + i * step[q] (i < count[q], host arrays)
 * of (dir, pt) ((3, ld) each, n rays) on the plane x = -a (coeffs_det[9] = a): num_steps points of
 * np.linspace(x_min, x_max), first argmin (NaN first, as np.argmin), range * shrink about it, until
 * tol > width > 1e-16 or max_attempts steps. d_out (device, (n_search, 4)): best_x, min_y, the last
 * x evaluated (compare_sep leaves it in coeffs_det[9]) and the final width. n_search <= 32,
 * num_steps <= 128. */
int akb_sep_search_f64(const double* dir, const double* pt, int64_t ld, int64_t n, int n_search,
                       const int64_t* h_start, const int64_t* h_step, const int64_t* h_count, double x_min,
                       double x_max, int num_steps, int max_attempts, double shrink, double tol, double* d_out,
                       void* stream);

/* Focus sweep rows (find_defocus, ref :9086-9170): for P detector planes x = -d_plane_j[p]
 * (coefficients g = 1, h = i = 0, j = d_plane_j[p], as coeffs_det[9] = -(s2f_middle + a)), the
 * hits of rays `subset` (m indices into the n rays; NULL = all, m = n) of (dir, pt), (3, ld) each.
 * d_sums == NULL: rows (2P, m) = [y_p0, z_p0, y_p1, ...]; else, with d_sums the pairwise sums of
 * those rows (akb_pairwise_sum_f64), rows = [(y - mean)^2, (z - mean)^2, ...], mean = sum / m
 * (np.std's two passes; sum the second rows again and divide by m for the variance). */
int akb_plane_sweep_rows_f64(const double* dir, const double* pt, int64_t ld, int64_t n, const int64_t* subset,
                             int64_t m, const double* d_plane_j, int P, const double* d_sums, double* rows,
                             void* stream);
/* The same two passes with np.std's sums fused (rays read once per pass, no rows written): plane p
 * feeds quantities 2p (y or (y - mean)^2) and 2p + 1 (z ...) of `sink` (nq = 2P rounded up to a
 * multiple of 16 - the extra quantities sum to 0 -, n = m, nan_mask 0); akb_leaf_finish_f64 then gives the numpy-order sums akb_pairwise_sum_f64 gives on
 * the rows. Pass B: d_sums = pass A's 2P sums. */
int akb_plane_sweep_sink_f64(const double* dir, const double* pt, int64_t ld, int64_t n, const int64_t* subset,
                             int64_t m, const double* d_plane_j, int P, const double* d_sums,
                             const akb_leaf_sink* sink, void* stream);

/* calc_dS (ref :13418-13473): area element of each point of a (V, H) grid of mirror points
 * (points (3, ld), flat index iv * H + ih): half the summed |cross| of the four neighbour
 * triangles, border points copied from the nearest interior point. V, H >= 3. */
int akb_calc_ds_f64(const double* points, int64_t ld, int V, int H, double* d_out, void* stream);

/* OPD maps (ref :3626, :3633, :3675-3677), with the means read from device memory as the tilt
 * sink left them (d_sum5 / d_cnt5 = sums and counts of det1_x, det1_y, det1_z, total1, total2;
 * mean = sum / count in float64):
 *   dist_err  = (total - mean_total) * 1e9
 *   sph       = ||det2 - mean_focus|| * 1e9
 *   wave      = dist_err2 - sph                                   (NULL outputs skipped)
 * d_extent_keys (optional, 4 x uint64): order-preserving keys of max(det2_y), -min(det2_y),
 * max(det2_z), -min(det2_z) over non-NaN rays (pupil pitch), zero-initialised by this call unless
 * keys_zeroed says the caller already zeroed them in stream order (akb_tilt_params_f64 does). */
int akb_opd_f64(const double* total1, const double* total2, const double* det2, int64_t ld, int64_t n,
                const double* d_sum5, const int64_t* d_cnt5, double* dist_err1, double* dist_err2,
                double* sph, double* wave, uint64_t* d_extent_keys, int keys_zeroed, void* stream);

/* Host function (no device work): the equal-angle resample between the two passes (ref
 * :2861-2870, KB_debug :11020-11030) for one axis, numpy / scipy 1.15 bit for bit:
 *   out = interp1d(angle_sep, rand, kind='linear')(np.linspace(angle_sep[0], angle_sep[-1], n))
 * angle_sep = np.arctan of the pass-1 exit slopes (taken by the caller with numpy), rand = the
 * pass-1 launch angles. AKB_E_INVALID with interp1d's message when a point is out of range. */
int akb_resample_f64(const double* angle_sep, const double* rand, int64_t n, double* out);

/* Wave2 (nm) of a shard (flat rays ray0 .. ray0 + nrays of the n x n grid) sampled onto a size x size
 * pupil in ray-index space (nearest ray, index (k * (n - 1)) // (size - 1)): opd_m[ky][kx] =
 * wave[iv * n + ih - ray0] * 1e-9 for the samples this shard owns, 0 elsewhere (shards are summed
 * across ranks: each sample has one owner, so the sum is exact). d_pitch (optional, device [2]):
 * (max y - min y) / (size - 1), (max z - min z) / (size - 1) from akb_opd_f64's extent keys. */
int akb_pupil_sample_f64(const double* wave, int64_t ray0, int64_t nrays, int64_t n, int size,
                         const uint64_t* d_extent_keys, double* opd_m, double* d_pitch, void* stream);

/* numpy-exact reduction: for each of `rows` rows of length n (row stride ld),
 * sum = the value np.sum gives (8192-element blocks, pairwise within a block, blocks added left
 * to right), count = number of summed elements. nan_to_zero=1 reproduces np.nansum/np.nanmean
 * (NaN -> 0, count excludes NaN). d_work: device scratch of akb_pairwise_work_bytes(rows, n).
 * Results: d_sum[rows], d_count[rows] (device). */
int64_t akb_pairwise_work_bytes(int rows, int64_t n);
int akb_pairwise_sum_f64(const double* x, int64_t ld, int rows, int64_t n, int nan_to_zero,
                         double* d_sum, int64_t* d_count, void* d_work, void* stream);

/* ---------------- Huygens-Fresnel phase accumulation ---------------- */

/* out[i] = sum_j u_j * exp(-i k r_ij) / r_ij,  r_ij = sqrt(((xi-xj)^2 + (yi-yj)^2) + (zi-zj)^2)
 * u_j = u_re_im[2j] + i u_re_im[2j+1] already multiplied by dS_j (ref CPU0402 :102).
 * out_re_im: interleaved complex128 (N).
 * splits: how many contiguous source ranges the sum is split over (0: the library's choice,
 * akb_huygens_splits). A target's sum is each range's partial (sources in order) and then the
 * partials summed in two ordered levels - chunks of 128 ranges, then the chunks - so it depends
 * only on m and the split count: run-to-run deterministic, and the same for any subset of targets
 * given the same split count (a target-sharded caller passes the whole problem's count). The
 * library's count depends on the device (its resident workgroups) and on n; it is capped so the
 * partials fit in 512 MiB.
 * work: device scratch of akb_huygens_work_bytes(n, m, splits) bytes: 16 n (splits + ceil(splits /
 * 128)) when splits > 1, at most ~516 MiB for the library's count (0 bytes for one split). One call
 * queues three kernels that use it: concurrent calls need their own work buffers. */
int akb_huygens_splits(int64_t n, int64_t m);
int64_t akb_huygens_work_bytes(int64_t n, int64_t m, int splits);
int akb_huygens_f64(const double* tx, const double* ty, const double* tz, int64_t n,
                    const double* sx, const double* sy, const double* sz, const double* u_re_im,
                    int64_t m, double k, double* out_re_im, int splits, void* work, void* stream);
/* u_out = u_in * ds (complex * real, ref CPU0402 :102 / GPU0402 :142) */
int akb_scale_field_f64(const double* u_re_im, const double* ds, int64_t m, double* out_re_im,
                        void* stream);

/* ---------------- PSF by FFT (rocFFT) ---------------- */

/* compute_psf_fft for a stack of `batch` wavelengths over one pupil:
 *   opd, amp: (ny, nx) float64 device arrays (NaN/inf -> 0); amp may be NULL, meaning
 *   amp = 1 where opd is finite and 0 elsewhere (psf_calc's mask, ref :1182-1188)
 *   d_pitch: optional device [dx, dy]; when given it replaces dx, dy (pitch computed on device)
 *   lambdas: host array of `batch` wavelengths
 *   hann_wy (ny) / hann_wx (nx) / hann_max: separable window or NULL (ref psf_fft.py:20-27)
 *   py = ny' * pad, px = nx' * pad with ny' = ny + ny%2 (ensure_even_size)
 *   psf: (batch, py, px) normalised intensity; efield_re_im: (batch, py, px) complex or NULL
 *   d_imax: device array of `batch` peak intensities before normalisation
 *   work: device scratch of akb_psf_work_bytes(...): for power-of-two pupils at pad 8 / 16 the
 *   line transforms' column-pass plane G (batch x nx' x py complex) plus per-row peak bookkeeping
 *   (row bounds, candidate rows: 16 bytes per psf row and batch entry); for other power-of-two
 *   pupils the pruned transform's plane; otherwise the padded field + rocFFT's work area.
 *   The peak max |F|^2 is exact on every route (AKB_PSF_PEAK = bound / f32 / f64 picks how its
 *   rows are searched; same bits). */
int64_t akb_psf_work_bytes(int ny, int nx, int pad, int batch);
int akb_psf_f64(const double* opd, const double* amp, int ny, int nx, int pad, int batch,
                const double* lambdas, double dx, double dy, const double* hann_wy,
                const double* hann_wx, double hann_max, double* psf, double* efield_re_im,
                double* d_imax, const double* d_pitch, void* work, void* stream);

/* ---------------- psf_calc pupil preparation (ref AKB_raytrace_20250312.py:1121-1188) ---------------- */

/* d_rows[c] = first row r with m[r][c] not NaN, -1 for an all-NaN column (the rotation
 * estimate's min_indices, :1122-1128; the caller forms rot with np.arctan as the reference). */
int akb_first_valid_rows_f64(const double* m, int ny, int nx, int32_t* d_rows, void* stream);

/* rotate_with_nan(m, angle, order=3) of psf_calc (:1138-1156): scipy.ndimage.rotate (reshape
 * False, mode 'constant', cubic B-spline) of the NaN-filled map and of its finite mask,
 * rotated = filled' / max(mask', 1e-12), NaN where mask' < 0.5. rot = [[c, s], [-s, c]] with
 * c = cosdg(angle), s = sindg(angle), offset = centre - rot @ centre (host-formed, as scipy
 * forms them); opd_m (optional) = rotated * 1e-9. work: akb_rotate_work_bytes(ny, nx). */
int64_t akb_rotate_work_bytes(int ny, int nx);
int akb_rotate_with_nan_f64(const double* m, int ny, int nx, const double rot[4], const double offset[2],
                            double* rotated, double* opd_m, void* work, void* stream);

/* ---------------- pupil-map post-processing (ref AKB_raytrace_20250312.py:9630-9693, legendre_fit.py:59-92) ---------------- */

/* The driver's whole chain from a gridded Wave2 map (ny * nx <= 65536) to compute_psf_fft's input
 * on the device, no host round trip (AKB_raytrace_20250312.py:3690-3700, :9630-9693,
 * :1121-1188): corrected = plane_correction_with_nan_and_outlier_filter(map - nanmean(map), sigma),
 * psf_calc's rotation estimate, rotated = rotate_with_nan(corrected, degrees(rot), order 3)
 * (cephes cosdg / sindg for scipy.ndimage.rotate's matrix), opd = rotated * 1e-9. Three launches:
 * the one-workgroup post, the B-spline prefilter (maps up to 128 x 128: one workgroup per array,
 * both axes in LDS), the rotation. work: akb_pupil_post_work_bytes(ny, nx). d_params (20 doubles):
 * nanmean, finite count, the quadratic fit (5), the plane (3), the outlier threshold, rot, its
 * degrees, cos, sin, the rotation's offset (2), error flags (bit 0: too few points for curve_fit,
 * bit 1: a singular normal system), nanmin and nanmax of the input map. Replaces
 * pupilmap._plane_corrections + psfcalc.rotation_estimate / rotate_with_nan where a pipelined
 * caller cannot wait on the host. */
int64_t akb_pupil_post_work_bytes(int ny, int nx);
int akb_pupil_post_f64(const double* map, int ny, int nx, double sigma, double* corrected, double* rotated,
                       double* opd, void* work, double* d_params, void* stream);

/* Sums for plane_correction_with_nan_and_outlier_filter (:9630) over the finite points of the
 * (ny, nx) map z, basis f = (1, X, Y, X^2, Y^2) with X = (2j - (nx-1))/(nx-1), Y likewise
 * (the reference's index coordinates, centred and scaled: the same least-squares fits).
 *   mode 0: normal equations of an nb-term fit (nb 3 or 5): d_out[0..14] upper triangle of
 *           sum f f^T (row-major, 5 x 5 slots), d_out[15..19] sum f z, d_out[20] count; with
 *           d_coef (5 terms) only points with |z - f.coef| < thr count (the 3-sigma filter).
 *   mode 1: d_out[0] = sum (z - f.coef), d_out[20] = count   (residual mean, :9672)
 *   mode 2: d_out[0] = sum (z - f.coef - mean)^2             (np.std of the residual, :9675)
 * The host solves the 5 x 5 / 3 x 3 systems. work: akb_moments_work_bytes(). Deterministic. */
int64_t akb_moments_work_bytes(void);
int akb_map_moments_f64(const double* z, int ny, int nx, int nb, const double* d_coef, double thr, int mode,
                        double mean, double* d_out, void* work, void* stream);
/* out = z - (c0 + c1 X + c2 Y), NaN kept (:9688-9691); d_coef3 on the device */
int akb_plane_subtract_f64(const double* z, int ny, int nx, const double* d_coef3, double* out, void* stream);

/* match_legendre_multi rows (legendre_fit.py:59-92) on an n x n map, K = order(order+1)/2
 * components with (ny, nx) = ord[2k], ord[2k+1]; px / py (order, n) the Legendre polynomials on
 * linspace(-1, 1, n) (host-evaluated with scipy.special.legendre, as the reference does).
 * mode 0: out[k] = Z_k * Z_k;  mode 1: out[k] = Z_k / sqrt(s[k]) * data;  mode 2: out[k] = c[k] * Z_k / sqrt(s[k]).
 * The nansums of modes 0 and 1 are akb_pairwise_sum_f64's rows (nan_mask 1). */
int akb_legendre_rows_f64(const double* data, int n, int K, int order, const double* px, const double* py,
                          const int* ord, const double* s, const double* c, int mode, double* out, void* stream);

/* ---------------- extract_affine_square_region (ref AKB_raytrace_20250312.py:1047-1119) ----------------
 * The reference uses OpenCV (absent from this image: parity with cv2 unpinned; these restate the
 * published algorithms as OpenCV 4.x implements them, see akb_affine_host.cpp).
 * akb_valid_mask_u8: mask = 255 where img is not NaN, else 0 (device).
 * akb_external_contours (HOST): cv2.findContours(mask, RETR_EXTERNAL, CHAIN_APPROX_SIMPLE) -
 *   contour c is xy[2 offsets[c] .. 2 offsets[c+1]) as (x, y) pairs, in cv2's order; fails with
 *   AKB_E_INVALID when the caller's capacities (cap points, ocap offsets) are too small, *n_xy and
 *   *n_contours still set.
 * akb_approx_poly_dp (HOST): cv2.approxPolyDP(src (count, 2) int32, eps, closed).
 * akb_affine_from_points (HOST): cv2.getAffineTransform(src[3] float32 pairs, dst[3]) -> M (2 x 3).
 * akb_affine_invert (HOST): M inverted as cv2.warpAffine does without WARP_INVERSE_MAP.
 * akb_warp_affine_f64: out (side x side) = cv2.warpAffine(nan_to_num(img), M, INTER_LINEAR),
 *   NaN where cv2.warpAffine(mask, M, INTER_NEAREST) == 0 (BORDER_CONSTANT 0); iM from
 *   akb_affine_invert (host array, passed by value). */
int akb_valid_mask_u8(const double* img, int ny, int nx, uint8_t* mask, void* stream);
int akb_external_contours(const uint8_t* mask, int rows, int cols, int64_t cap, int32_t* xy, int64_t* n_xy,
                          int32_t ocap, int32_t* offsets, int32_t* n_contours);
int akb_approx_poly_dp(const int32_t* src, int32_t count, double eps, int closed, int32_t* dst, int32_t* n_out);
int akb_affine_from_points(const float* src, const float* dst, double* M);
int akb_affine_invert(const double* M, double* iM);
int akb_warp_affine_f64(const double* img, int ny, int nx, const double* iM, int side, double* out, void* stream);

/* ---------------- griddata(method='cubic') on the ray grid (ref AKB_raytrace_20250312.py:3673, :3689) ----------------
 * scipy's Clough-Tocher griddata for points that are the n_v x n_h ray grid's detector hits
 * (x = detcenter2[1], y = detcenter2[2], ray iv * n_h + ih) onto the meshgrid of gx x gy.
 * Triangulation: akb_gd_cells_f64 (cell diagonals by the in-circle test, checks; flags bit 0
 * non-convex cell, bit 1 not locally Delaunay, bit 2 broken pocket adjacency, bits 3 and 4 both
 * set = folded grid) -> akb_gd_pockets (HOST: the triangles between the boundary ring and the
 * convex hull, ring coordinates from akb_gd_cells_f64; ids >= 2 (n_v-1)(n_h-1)) ->
 * akb_gd_check_pockets. Gradients: akb_gd_grad_sweeps_f64 (Chebyshev-accelerated Jacobi sweeps of
 * scipy's estimate_gradients_2d_global local solve, in the edge-matrix form g <- c - P S with
 * S = sum over the edges of r^-3 e e^T g_j; the largest relative change of each Jacobi step
 * atomically max-ed into d_change as double bits) until converged. Values: akb_gd_eval_f64 (NaN
 * outside the hull). */
int akb_gd_cells_f64(const double* x, const double* y, int nv, int nh, uint8_t* diag, double tol, unsigned* d_flags,
                     double* ring_x, double* ring_y, void* stream);
int akb_gd_pockets(const double* ring_x, const double* ring_y, int nv, int nh, int cap, int32_t* n_out,
                   int32_t* tri, int32_t* nbr, int32_t* edge_tri, int32_t* extra_ptr, int32_t* extra_idx);
int akb_gd_check_pockets(const double* x, const double* y, int nv, int nh, const uint8_t* diag, int npock,
                         const int32_t* ptri, const int32_t* pnbr, const int32_t* edge_tri, double tol,
                         unsigned* d_flags, void* stream);
/* kk = 1 or 2 sweeps in one launch (register kernel, wave-shift neighbours, the second sweep one row
 * behind the first): gout1 = x_{k+1}, gout2 = x_{k+2} from gin = x_k (NULL: zeros) and gprev =
 * x_{k-1} (NULL: the first sweep is plain), Chebyshev weights om1, om2 (x_{k+1} = om (y - x_{k-1}) +
 * x_{k-1}, y the Jacobi step). d_change[0..kk-1]: the sweeps' changes; ring_work: 22 * ring-length
 * doubles. Replaces the gradient loop of scipy/interpolate/_interpnd.pyx. */
int akb_gd_grad_sweeps_f64(const double* x, const double* y, int nv, int nh, const uint8_t* diag, int npock,
                           const int32_t* ptri, const int32_t* pnbr, const int32_t* edge_tri, const int32_t* xptr,
                           const int32_t* xidx, const double* f, int nvals, const double* gin, const double* gprev,
                           double om1, double om2, int kk, double* gout1, double* gout2, double* ring_work,
                           unsigned long long* d_change, void* stream);
int akb_gd_eval_f64(const double* x, const double* y, int nv, int nh, const uint8_t* diag, int npock,
                    const int32_t* ptri, const int32_t* pnbr, const int32_t* edge_tri, const double* gx, int mx,
                    const double* gy, int my, const double* f, const double* grad, int nvals, int* owner,
                    double* out, void* stream);

/* The same interpolation with the gradients of exactly K Chebyshev sweeps (1 <= K <= 14, omegas[j]
 * the weight of sweep j + 1 as CubicGrid.gradients forms them), computed only where the targets
 * read them: per interior target cell a (2K + 4)^2 patch in LDS, the global iteration on the
 * boundary band (depth 2K + 2, pocket chords included) for the rest. The values equal
 * akb_gd_eval_f64 on the global iteration's K-sweep gradients bit for bit; one call, no host
 * synchronisation. work: akb_gd_cone_work_bytes; d_change (or NULL, 2 words, ordered double bits,
 * atomic max): [0] the largest change measure (scipy's) one more sweep would make at the interior
 * target cells' corners, [1] the largest value-error estimate of an interior target cell (2 sqrt 2 x
 * the corners' largest |one more plain sweep - x_K| x the cell's longest side or diagonal: the map
 * units' bound on |value - the converged iteration's value| with the Jacobi spectrum in [-1/2, 1/2]),
 * maxed with the boundary-band and pocket targets' own estimate (twice the value change one more plain
 * band sweep makes there, k_gd_eval; a NaN estimate is stored as +inf). Replaces the gradient loop of scipy's
 * estimate_gradients_2d_global
 * (scipy/interpolate/_interpnd.pyx) where the driver's griddata (AKB_raytrace_20250312.py:3689)
 * feeds a fixed-size pupil. */
int64_t akb_gd_cone_work_bytes(int nv, int nh, int mx, int my, int nvals);
/* Diagnostics of the cone solve's patch kernel (k_gd_cone_patch), for bench.py's roofline:
 * akb_gd_patch_timing(1) records HIP events around every patch launch from then on (the last 1024
 * launches kept; 0 stops and keeps the record, 1 starts a new one; 2 also clocks every band sweep
 * workgroup - device atomics in each, which lengthen the step: never inside a timed region);
 * akb_gd_patch_times waits for them and writes up
 * to max launch durations (ms, oldest first) and, when cells != NULL, each launch's interior target
 * cell count; returns how many (or a negative AKB error code). */
int akb_gd_patch_timing(int enable);
int akb_gd_patch_times(float* ms, int* cells, int max);
/* the same record of the boundary band's sweeps: one duration (ms) per value set's band iteration
 * (the K sweep launches and the guard's extra sweep, events around all of them) */
int akb_gd_band_times(float* ms, int max);
/* while timing (100 MHz wall-clock ticks, summed over the launches since akb_gd_patch_timing(1);
 * waits for the device), out[0..9]: the patch kernel's workgroup 0 in its steps' phases - the
 * setup (box in, vertex constants), the sweeps, the rest (corners, next box) - and its step count;
 * the band sweeps' ring-only workgroups' time and count, their workgroups with a tile (and a share
 * of the ring) time and count, the longest of each */
int akb_gd_patch_phases(unsigned long long* out);
/* The patch kernel's thread -> box vertex table for K sweeps (host only, no device call): out[t] =
 * r | c << 8 of thread t's vertex in the (2K + 4)^2 box, 0xffff for the corner-store and idle
 * threads; writes 1024 entries and returns the kernel's split S (the thread sets: inner A = [0, N2),
 * inner B = [N2, 2 N2), outer = [2 N2, N1 + N2) with N1 = (2K + 2)^2, N2 = (2K + 2 - 2S)^2), or a
 * negative AKB error code for K outside 1 .. 14. */
int akb_gd_patch_order(int K, uint16_t* out);
/* The driver's target axes (AKB_raytrace_20250312.py:3654-3657): gx = np.linspace(min, max, mx) of
 * the lattice's x (its extremes lie on the boundary ring akb_gd_cells_f64 returns), gy likewise of
 * y; d_extent (or NULL, 6 doubles): [min x, max x, min y, max y, dx, dy] with dx = |gh[0,1] - gh[0,0]|,
 * dy = |gv[1,0] - gv[0,0]| of the meshgrids after the driver's grid_H -= np.mean(grid_H) (numpy's
 * pairwise mean; :3698): the pupil pitch psf_calc hands compute_psf_fft (:1176-1177). One
 * workgroup, device-resident. */
int akb_gd_axes_f64(const double* ring_x, const double* ring_y, int64_t L, int mx, int my, double* gx, double* gy,
                    double* d_extent, void* stream);
int akb_gd_cone_eval_f64(const double* x, const double* y, int nv, int nh, const uint8_t* diag, int npock,
                         const int32_t* ptri, const int32_t* pnbr, const int32_t* edge_tri, const int32_t* xptr,
                         const int32_t* xidx, const double* gx, int mx, const double* gy, int my, const double* f,
                         int nvals, int K, const double* omegas, void* work, int* owner, double* out,
                         unsigned long long* d_change, void* stream);
/* The one-process cone solve split at the pockets (FaithfulPupil's begin / finish): the axes from
 * the ring first (akb_gd_ring_f64 + akb_gd_axes_f64), then
 *   akb_gd_cells_claims_f64: akb_gd_cells_f64's cell pass (the same diag and flags; no ring) with
 *     the cells' target claims fused in: owner[] = INT32_MAX, then each 16 x 16 tile of cells
 *     whose vertex box can hold a target claims from its LDS copy (the same owners as the claims
 *     of akb_gd_cone_eval_f64);
 *   akb_gd_claim_pockets_f64: the pocket triangles' claims into those owners (atomicMin);
 *   akb_gd_cone_solve_f64: akb_gd_cone_eval_f64 on the claimed owners (no claims of its own).
 * Every target value is akb_gd_cone_eval_f64's bit for bit. */
int akb_gd_cells_claims_f64(const double* x, const double* y, int nv, int nh, uint8_t* diag, double tol,
                            unsigned* d_flags, const double* gx, int mx, const double* gy, int my, int* owner,
                            void* stream);
int akb_gd_claim_pockets_f64(const double* x, const double* y, int nv, int nh, const uint8_t* diag, int npock,
                             const int32_t* ptri, const double* gx, int mx, const double* gy, int my, int* owner,
                             void* stream);
int akb_gd_cone_solve_f64(const double* x, const double* y, int nv, int nh, const uint8_t* diag, int npock,
                          const int32_t* ptri, const int32_t* pnbr, const int32_t* edge_tri, const int32_t* xptr,
                          const int32_t* xidx, const double* gx, int mx, const double* gy, int my, const double* f,
                          int nvals, int K, const double* omegas, void* work, const int* owner, double* out,
                          unsigned long long* d_change, void* stream);

/* The cone solve of a lattice sharded over ranks (row-block shards of the flat ray index; each
 * rank passes x, y, diag as "virtual" global arrays of which only its rows plus K + 3 halo rows are
 * backed - pointer minus row0 * nh - and the band owner passes full arrays with the boundary band
 * filled):
 *   akb_gd_cells_window_f64: the cell pass over cell rows [row0, row1) (no ring);
 *   akb_gd_ring_f64: the boundary ring's coordinates (the band owner, for the host pockets);
 *   akb_gd_claims_f64: owner[] = INT32_MAX, then the claims of the cells in rows [row0, row1)
 *     (row1 < 0: all) and, with with_pockets, of the pocket triangles; a MIN all-reduce of the
 *     ranks' owners gives the one-process owners (the same atomicMin over all triangles); work
 *     (or NULL): an akb_gd_cone_work_bytes(nv, nh, mx, my, 1) buffer for the block scan's flags;
 *   akb_gd_cone_part_f64: with that global owner, the targets this rank forms - interior cells
 *     whose p00 lies in its rays [own0, own1), and with band_on every band / pocket target - their
 *     gradients and values: out (nvals, my, mx) and cnt (my, mx) hold value / 1 there, 0 elsewhere,
 *     so a SUM reduction of the ranks' pieces assembles the map;
 *   akb_gd_part_finish_f64: NaN where the reduced cnt is 0 (outside the hull).
 * Every target value is the one-process akb_gd_cone_eval_f64's bit for bit. */
int akb_gd_cells_window_f64(const double* x, const double* y, int nv, int nh, int row0, int row1, uint8_t* diag,
                            double tol, unsigned* d_flags, void* stream);
int akb_gd_ring_f64(const double* x, const double* y, int nv, int nh, double* ring_x, double* ring_y, unsigned* d_flags,
                    void* stream);
int akb_gd_claims_f64(const double* x, const double* y, int nv, int nh, const uint8_t* diag, int npock,
                      const int32_t* ptri, const int32_t* pnbr, const int32_t* edge_tri, int row0, int row1,
                      int with_pockets, const double* gx, int mx, const double* gy, int my, int* owner, void* work,
                      void* stream);
int akb_gd_cone_part_f64(const double* x, const double* y, int nv, int nh, const uint8_t* diag, int npock,
                         const int32_t* ptri, const int32_t* pnbr, const int32_t* edge_tri, const int32_t* xptr,
                         const int32_t* xidx, int64_t own0, int64_t own1, int band_on, const double* gx, int mx,
                         const double* gy, int my, const double* f, int nvals, int K, const double* omegas, void* work,
                         const int* owner, double* out, double* cnt, unsigned long long* d_change, void* stream);
int akb_gd_part_finish_f64(double* out, const double* cnt, int64_t m, int nvals, void* stream);

/* diagnostics: out[13i..13i+12] = (the trace's sqrt, sqrt, the trace's shared-reciprocal a/b, a/b,
 * the positive-divisor a/b, the trace's norm and reciprocal norm of (a, b, b), sqrt and 1/sqrt of
 * that squared norm, the trace's slope arctan of a, the library atan of a, the trace's a/b and
 * 1/b) for n pairs (a[i], b[i]) — used by the tests to check the shortcuts bit for bit (the
 * arctan to its stated accuracy) */
#define AKB_SELFTEST_COLS 13
int akb_selftest_arith_f64(const double* a, const double* b, int64_t n, double* out, void* stream);

/* release the cached rocFFT plans (and rocFFT itself) and the device twiddle tables */
void akb_psf_release_plans(void);

/* release every device / pinned resource the library caches between calls - rocFFT plans and
 * twiddle tables, the staged-argument ring's pinned buffers and events, the patch-timing events -
 * while the HIP runtime is still up (bindings call it from an exit hook: the Python package's
 * atexit). No HIP call is made for a cache that was never filled; the library stays usable */
void akb_release_all(void);

#ifdef __cplusplus
}
#endif

#endif /* AKB_RAYTRACE_H */
