/*
 * mfnerf.h -- C ABI of libmfnerf_hip.so, the MI355X (gfx950) kernels behind MF-NeRF's
 * volumetric-rendering training step.
 *
 * Conventions (every entry point):
 *   - plain device pointers + sizes, row-major contiguous arrays, no torch types;
 *   - the last argument is the HIP stream the work is enqueued on (NULL = legacy default);
 *   - return 0 on success, a nonzero MFN_ERR_* code otherwise; mfnerf_last_error()
 *     returns a message for the calling thread's last failure;
 *   - no entry point allocates, frees or synchronises: callers pass workspace, so every
 *     call is legal inside hipStreamBeginCapture (HIP graphs);
 *   - outputs are NOT pre-zeroed by the library unless stated ("zero-fills").
 *
 * Reference interfaces replaced (lly00412/MF-NeRF, paths relative to the repo root):
 *   vren pybind module: models/csrc/binding.cpp:234-250 (C++ signatures binding.cpp:4-231,
 *   models/csrc/include/utils.h:9-126); tiny-cuda-nn HashGrid / SphericalHarmonics /
 *   FullyFusedMLP as configured in models/networks.py:36-79; apex FusedAdam (train.py:136).
 */
#ifndef MFNERF_H
#define MFNERF_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* mfnerf_stream_t; /* == hipStream_t */

#define MFN_OK 0
#define MFN_ERR_INVALID 1 /* bad argument (null pointer, bad size, unsupported config) */
#define MFN_ERR_LAUNCH 2  /* HIP launch error */

const char* mfnerf_last_error(void);
int mfnerf_abi_version(void);

/* Mixed-precision state of a training step, device-resident (32 bytes, zero-initialised by the
 * caller, then scale / growth_interval / growth_factor / backoff_factor set): torch.cuda.amp.GradScaler
 * as PyTorch-Lightning's precision=16 drives it (train.py:287; init scale 65536, growth 2.0 every
 * 2000 clean steps, backoff 0.5).  Producers of the step's gradient raise `nonfinite`; the optimizer
 * call skips the update when it is set and then runs GradScaler.update() on the device.
 * growth_interval == 0: static scaling (the skip only; mfnerf_field_bw then uses its grad_scale). */
typedef struct {
    int32_t nonfinite;       /* 1 when some gradient of the step is inf/nan; cleared by the optimizer */
    int32_t skipped;         /* optimizer steps skipped so far */
    float scale;             /* current loss scale (dynamic mode) */
    int32_t growth_tracker;  /* clean steps since the last scale change */
    int32_t growth_interval; /* 2000; 0 = static */
    float growth_factor;     /* 2.0 */
    float backoff_factor;    /* 0.5 */
    int32_t ticket;          /* the optimizer pass's last-workgroup ticket; 0 between calls */
} mfnerf_amp_state;

/* ---------------------------------------------------------------- vren ops */

/* vren.ray_aabb_intersect (binding.cpp:4-16, intersection.cu:59-100).
 * rays_o, rays_d (n_rays,3) f32; centers, half_sizes (n_voxels,3) f32.
 * Writes hit_cnt (n_rays) i32, hits_t (n_rays,max_hits,2) f32, hits_voxel_idx (n_rays,max_hits) i64;
 * zero-fills / -1-fills all three.  Hits are kept in voxel order and sorted near->far by t1. */
int mfnerf_ray_aabb_intersect(const float* rays_o, const float* rays_d, const float* centers,
                              const float* half_sizes, int64_t n_rays, int64_t n_voxels, int max_hits,
                              int32_t* hit_cnt, float* hits_t, int64_t* hits_voxel_idx, mfnerf_stream_t stream);

/* vren.morton3D (binding.cpp:46-50, raymarching.cu:62-88): coords (n,3) i32 -> out (n) i32. */
int mfnerf_morton3d(const int32_t* coords, int64_t n, int32_t* out, mfnerf_stream_t stream);

/* vren.morton3D_invert (binding.cpp:53-57, raymarching.cu:90-119): idx (n) i32 -> coords (n,3) i32. */
int mfnerf_morton3d_invert(const int32_t* idx, int64_t n, int32_t* coords, mfnerf_stream_t stream);

/* vren.packbits (binding.cpp:34-43, raymarching.cu:122-161): bit i of byte n = grid[8n+i] > thr.
 * grid (8*n_bytes) f32.  thr_dev, when non-NULL, is a device f32 read instead of `thr`
 * (keeps the occupancy update free of host syncs). */
int mfnerf_packbits(const float* grid, int64_t n_bytes, float thr, const float* thr_dev, uint8_t* bitfield,
                    mfnerf_stream_t stream);

/* Workspace bytes mfnerf_raymarching_train needs for n_rays rays of at most max_samples samples
 * (the per-ray counts, and the march's per-ray sample positions t: n_rays x max_samples f32). */
int64_t mfnerf_raymarching_train_workspace(int64_t n_rays, int max_samples);

/* vren.raymarching_train (binding.cpp:60-85, raymarching.cu:166-332).
 * hits_t: (n_rays,2) f32 rows (t1,t2) with row stride hits_stride floats.
 * Outputs: rays_a (n_rays,3) i64 -- row r = (r, start, count), start = exclusive prefix sum
 *          (canonical order; the reference's atomicAdd order is nondeterministic);
 *          xyzs, dirs (capacity,3), deltas, ts (capacity) f32 -- samples [0, counter[0]);
 *          counter (2) i32 = (total samples, n_rays).  Samples beyond `capacity` are dropped
 *          (their rays' counts are clipped).  Device-resident count: no host sync. */
int mfnerf_raymarching_train(const float* rays_o, const float* rays_d, const float* hits_t, int64_t hits_stride,
                             const uint8_t* bitfield, int cascades, float scale, float exp_step_factor,
                             const float* noise, int grid_size, int max_samples, int64_t n_rays, int64_t capacity,
                             int64_t* rays_a, float* xyzs, float* dirs, float* deltas, float* ts, int32_t* counter,
                             void* workspace, mfnerf_stream_t stream);

/* vren.raymarching_test (binding.cpp:88-115, raymarching.cu:335-454), including the reference's
 * calc_dt(..., cascades) quirk.  hits_t (n_rays,2 with row stride hits_stride) is updated in place
 * (column 0).  Zero-fills xyzs, dirs (n_alive,N_samples,3), deltas, ts (n_alive,N_samples), n_eff (n_alive) i32. */
int mfnerf_raymarching_test(const float* rays_o, const float* rays_d, float* hits_t, int64_t hits_stride,
                            const int64_t* alive_indices, int64_t n_alive, const uint8_t* bitfield, int cascades,
                            float scale, float exp_step_factor, int grid_size, int max_samples, int N_samples,
                            float* xyzs, float* dirs, float* deltas, float* ts, int32_t* n_eff,
                            mfnerf_stream_t stream);

/* vren.composite_train_fw (binding.cpp:118-136, volumerendering.cu:6-84).
 * sigmas (n_samples), rgbs (n_samples,3), deltas, ts f32; rays_a (n_rays,3) i64.
 * Writes total_samples (indexed by ray id) i64, opacity, depth (n_rays), rgb (n_rays,3) and ws for every
 * sample of every listed ray (0 after the ray terminates); no memset of n_samples-sized buffers. */
int mfnerf_composite_train_fw(const float* sigmas, const float* rgbs, const float* deltas, const float* ts,
                              const int64_t* rays_a, int64_t n_rays, int64_t n_samples, float T_threshold,
                              int64_t* total_samples, float* opacity, float* depth, float* rgb, float* ws,
                              mfnerf_stream_t stream);

/* vren.composite_train_bw (binding.cpp:139-173, volumerendering.cu:87-202).  Writes dL_dsigmas (n_samples)
 * and dL_drgbs (n_samples,3) for every sample of every listed ray (0 after the ray terminates).
 * The per-ray scan of dL_dws*ws (host-side + thrust in the reference) is done in-kernel. */
int mfnerf_composite_train_bw(const float* dL_dopacity, const float* dL_ddepth, const float* dL_drgb,
                              const float* dL_dws, const float* sigmas, const float* rgbs, const float* ws,
                              const float* deltas, const float* ts, const int64_t* rays_a, const float* opacity,
                              const float* depth, const float* rgb, int64_t n_rays, int64_t n_samples,
                              float T_threshold, float* dL_dsigmas, float* dL_drgbs, mfnerf_stream_t stream);

/* Fused training compositing for the default loss (no distortion term): mfnerf_composite_train_fw,
 * mfnerf_nerf_loss (target, n_mean, lambda_opacity, bg) and mfnerf_composite_train_bw with
 * dL_ddepth = 0, dL_dws = 0 in one pass (one wave per ray); the same outputs as the three calls,
 * bit-identical.  loss_partials (optional, ceil(n_rays/4) device f32) is OVERWRITTEN with the loss
 * value as one partial sum per 4 rays (their sum is the loss; no zeroing needed).  Replaces the chain at rendering.py:121-163 + losses.py:47-60
 * + custom_functions.py:148-159 in one training step. */
int mfnerf_composite_train_fused(const float* sigmas, const float* rgbs, const float* deltas, const float* ts,
                                 const int64_t* rays_a, int64_t n_rays, int64_t n_samples, float T_threshold,
                                 const float* target, int64_t n_mean, float lambda_opacity, float bg_r, float bg_g,
                                 float bg_b, int64_t* total_samples, float* opacity, float* depth, float* rgb,
                                 float* ws, float* dL_drgb, float* dL_dopacity, float* dL_dsigmas, float* dL_drgbs,
                                 float* loss_partials, mfnerf_stream_t stream);

/* vren.composite_test_fw (binding.cpp:176-201, volumerendering.cu:205-285).  sigmas (n_alive,N_samples),
 * rgbs (n_alive,N_samples,3), deltas, ts (n_alive,N_samples); in place on alive_indices, opacity,
 * depth, rgb (indexed by ray). */
int mfnerf_composite_test_fw(const float* sigmas, const float* rgbs, const float* deltas, const float* ts,
                             int64_t* alive_indices, int64_t n_alive, int N_samples, float T_threshold,
                             const int32_t* n_eff, float* opacity, float* depth, float* rgb,
                             mfnerf_stream_t stream);

/* vren.distortion_loss_fw (binding.cpp:204-216, losses.cu:9-109).  Zero-fills loss (n_rays) and
 * writes ws_inclusive_scan, wts_inclusive_scan (n_samples). */
int mfnerf_distortion_loss_fw(const float* ws, const float* deltas, const float* ts, const int64_t* rays_a,
                              int64_t n_rays, int64_t n_samples, float* loss, float* ws_incl, float* wts_incl,
                              mfnerf_stream_t stream);

/* vren.distortion_loss_bw (binding.cpp:219-231, losses.cu:112-175).  Zero-fills dL_dws (n_samples). */
int mfnerf_distortion_loss_bw(const float* dL_dloss, const float* ws_incl, const float* wts_incl,
                              const float* ws, const float* deltas, const float* ts, const int64_t* rays_a,
                              int64_t n_rays, int64_t n_samples, float* dL_dws, mfnerf_stream_t stream);

/* NeRFLoss (losses.py:47-60) + the background blend (rendering.py:153-161) and its gradient, fused:
 * pred = rgb + bg*(1-opacity); loss = mean((pred-target)^2) + lambda_opacity*mean(-o ln o),
 * o = opacity+1e-10 (train.py:178 sums the two means).  Writes dL_drgb (n,3), dL_dopacity (n);
 * loss_sum (optional, device f32) is ACCUMULATED with the loss value.  n_mean: the ray count the
 * means are taken over (0 = n_rays); a batch computed in parts passes the full batch size so the
 * parts' losses and gradients add up to the whole batch's. */
int mfnerf_nerf_loss(const float* rgb, const float* opacity, const float* target, int64_t n_rays, int64_t n_mean,
                     float lambda_opacity, float bg_r, float bg_g, float bg_b, float* dL_drgb, float* dL_dopacity,
                     float* loss_sum, mfnerf_stream_t stream);

/* ---------------------------------------------------------------- grid encoding (tcnn HashGrid / MF) */

/* Level table of a multiresolution grid (tcnn GridEncodingTemplated, networks.py:39-49).
 * Host-computed once; per level: scale = exp2f(l*log2f(b))*N_min - 1, res = ceil(scale)+1,
 * offset/size in entries (of n_features values each).  table_kind: 0 own table (dense when
 * res^3 <= size, else coherent prime hash), 1 MixedFeature shared table (canonical-grid index). */
#define MFN_MAX_LEVELS 32
typedef struct {
    int32_t n_levels;
    int32_t n_features;         /* F: only 2 is supported by the kernels */
    int32_t canon_res;          /* MixedFeature canonical grid resolution */
    int32_t pad_;
    float scale[MFN_MAX_LEVELS];
    uint32_t res[MFN_MAX_LEVELS];
    uint32_t offset[MFN_MAX_LEVELS];
    uint32_t size[MFN_MAX_LEVELS];
    int32_t table_kind[MFN_MAX_LEVELS];
} mfnerf_grid_desc;

/* Encode points x (n,3) f32.  The kernel first normalises x' = (x - x_min) / x_range exactly as
 * NGP.density does in torch (networks.py:105: (x-xyz_min)/(xyz_max-xyz_min); pass 0, 1 for inputs
 * already in [0,1]^3).  table (n_entries*F) f16.  out (n, n_levels*F) f16 row-major.
 * n_dev (optional, device i32): live row count <= n (rows beyond it are skipped). */
int mfnerf_grid_encode_fw(const float* x, int64_t n, const int32_t* n_dev, float x_min, float x_range,
                          const mfnerf_grid_desc* desc, const void* table_f16, void* out_f16,
                          mfnerf_stream_t stream);

/* mfnerf_grid_encode_fw with a level-major output: out_planes (n_levels, plane_stride) half2, the
 * features of level l of point i at [l*plane_stride + i] (plane_stride >= n).  Work is split by
 * level over the 8 XCDs so each XCD's L2 holds only its levels' tables. */
int mfnerf_grid_encode_fw_planar(const float* x, int64_t n, const int32_t* n_dev, float x_min, float x_range,
                                 const mfnerf_grid_desc* desc, const void* table_f16, void* out_planes,
                                 int64_t plane_stride, mfnerf_stream_t stream);

/* Scatter dL/dout (n, n_levels*F) f32 into grad_table (n_entries*F) f32.  workspace (optional,
 * mfnerf_grid_encode_bw_workspace() bytes, ZERO on the first call; the call leaves it zero again):
 * private copies of the dense coarse levels' gradient, which spread their hot-line atomics.
 * level_l1 == NULL: float atomics, ACCUMULATES into grad_table (caller zeroes).
 * level_l1 != NULL (device f32[n_levels] = mfnerf_grid_level_l1 of dL_dout, or any upper bound of
 * it): fixed-point accumulation -- int32 atomics of rint(v * 2^(30-e_l)), l1_l < 2^e_l, which cannot
 * overflow and run ~28% faster than float atomics on MI355X -- then converted back; grad_table must
 * be ZERO on entry and is OVERWRITTEN.  Resolution per level 2^(e_l-30) (~1e-9 of the level's L1). */
int64_t mfnerf_grid_encode_bw_workspace(const mfnerf_grid_desc* desc);
int mfnerf_grid_encode_bw(const float* x, int64_t n, const int32_t* n_dev, float x_min, float x_range,
                          const mfnerf_grid_desc* desc, const float* dL_dout, float* grad_table, void* workspace,
                          const float* level_l1, mfnerf_stream_t stream);

/* mfnerf_grid_encode_bw in two calls (the scatter, then the fold of the private copies /
 * fixed-point conversion), so the scatter can be timed on its own and the finish scheduled later
 * (anything reading grad_table must come after the finish). */
int mfnerf_grid_encode_bw_scatter(const float* x, int64_t n, const int32_t* n_dev, float x_min, float x_range,
                                  const mfnerf_grid_desc* desc, const float* dL_dout, float* grad_table,
                                  void* workspace, const float* level_l1, mfnerf_stream_t stream);
int mfnerf_grid_encode_bw_finish(const mfnerf_grid_desc* desc, float* grad_table, void* workspace,
                                 const float* level_l1, mfnerf_stream_t stream);

/* The fixed-point scatter (level_l1 required) by table partitions instead of memory-side atomics:
 * the hashed / shared tables are cut into partitions of up to 2048 entries; every (point, level,
 * corner row) becomes an 8-B record, sorted by partition in LDS and stored into fixed per-(partition,
 * work unit) slots, and one workgroup per partition sums its records exactly (int64 LDS atomics)
 * and stores the partition once, rounded to the same int32 fixed point as
 * mfnerf_grid_encode_bw_scatter (one rounding per entry).  parts: 1 = the dense coarse levels only
 * (atomics into the workspace's private copies, as mfnerf_grid_encode_bw_scatter), 2 = the
 * partitioned levels only, 3 = both.  The workspace prefix is the private copies, so
 * mfnerf_grid_encode_bw_finish / mfnerf_adam_step_fixed convert the result unchanged; grad_table must
 * be zero on entry before the partitioned tables (the levels added by atomics), and is overwritten
 * from there on.  workspace: mfnerf_grid_encode_bw_binned_workspace(desc, n_slots) bytes, zero on the
 * first call (the finish and the accumulate leave it zero); n_slots (0 or > n: n) is the live sample
 * count the record slots are sized for -- a training step passes its expected count, not its
 * capacity (rays x 1024 samples): a live count well above n_slots overflows slots, whose extra
 * records are added by integer atomics into the workspace's overflow words and from there into the
 * partition's sums (same sums, slower).  Bit-reproducible.  Replaces tcnn's hash-grid backward
 * scatter (networks.py:36-49 encoding, half2 atomics there). */
int64_t mfnerf_grid_encode_bw_binned_workspace(const mfnerf_grid_desc* desc, int64_t n_max);
/* Adam arguments for the fused partitioned accumulate (mfnerf_grid_encode_bw_binned_adam). */
typedef struct {
    float* params;            /* the flat f32 master parameters, Adam m and v, and the f16 mirror */
    float* m;
    float* v;
    void* p16;
    int64_t table_offset;     /* index of the grid table's first value in those vectors */
    float lr, beta1, beta2, eps;
    const int32_t* step_dev;  /* as mfnerf_adam_step_fixed */
    const float* lr_dev;
    const mfnerf_amp_state* amp;
} mfnerf_adam_fused;
int mfnerf_grid_encode_bw_binned(const float* x, int64_t n, const int32_t* n_dev, float x_min, float x_range,
                                 const mfnerf_grid_desc* desc, const float* dL_dout, float* grad_table,
                                 void* workspace, int64_t n_slots, const float* level_l1, int parts,
                                 mfnerf_stream_t stream);
/* mfnerf_grid_encode_bw_binned (parts = 3) + mfnerf_grid_encode_bw_finish in float form for an
 * exchange before the optimizer (the data-parallel step): the accumulate writes the partitioned
 * tables' finished sums as floats (times 1 / the table's scale, as the finish would) and one finish
 * pass covers only the values before them.  Same floats as the two-call form.  grad_table must be
 * zero before the partitioned tables' first value (mfnerf_grid_binned_first_value); the rest is
 * overwritten.  Replaces tcnn's hash-grid backward (networks.py:36-49) feeding DDP's all-reduce
 * (train.py:284).  gate (optional, mfnerf_gate_wait): signalled once as the dense-level launch
 * starts (by its first workgroup; a signal launch when no dense-level launch runs).
 * flag (optional): mfnerf_flag_to_shards(grads, flag_world, flag_shard_len, flag) folded into the
 * finish pass, grad_table being grads + table_offset (the flat gradient's every value must be final
 * when this is enqueued; needs a non-empty table prefix before the partitioned tables). */
int mfnerf_grid_encode_bw_binned_float(const float* x, int64_t n, const int32_t* n_dev, float x_min, float x_range,
                                       const mfnerf_grid_desc* desc, const float* dL_dout, float* grad_table,
                                       void* workspace, int64_t n_slots, const float* level_l1, int32_t* gate,
                                       const int32_t* flag, int64_t flag_world, int64_t flag_shard_len,
                                       int64_t table_offset, mfnerf_stream_t stream);
/* mfnerf_grid_encode_bw_binned (parts = 3) with the partitioned tables' Adam step fused into the
 * accumulate (adam: see mfnerf_adam_step_fixed_partial). */
int mfnerf_grid_encode_bw_binned_adam(const float* x, int64_t n, const int32_t* n_dev, float x_min, float x_range,
                                      const mfnerf_grid_desc* desc, const float* dL_dout, float* grad_table,
                                      void* workspace, int64_t n_slots, const float* level_l1,
                                      const mfnerf_adam_fused* adam, mfnerf_stream_t stream);
/* The collective-free step's whole table-gradient + optimizer tail in three launches: the binned
 * scatter (parts = 3), an accumulate launch whose partitions apply Adam to the partitioned tables
 * (as mfnerf_grid_encode_bw_binned_adam) while its leading workgroups run mfnerf_adam_step_fixed's
 * update over [0, the partitioned tables' first value) -- the MLPs and the dense levels, whose
 * gradients are final before the scatter -- and a last small pass for the step's bookkeeping (step
 * count, GradScaler, level_l1 zeroed).  grads: the flat gradient of n_params values (the table's
 * at adam->table_offset), zero for the table on entry; step_dev / amp: adam's, writable.  Same bits
 * as mfnerf_grid_encode_bw_binned_adam + mfnerf_adam_step_fixed_partial (and as the unfused
 * mfnerf_grid_encode_bw_binned + mfnerf_adam_step_fixed).  packed (optional, else NULL): the last pass
 * also repacks the MLP weights from adam->p16 into the field head's fragment blob for rgb width
 * rgb_width (= mfnerf_field_pack_weights_f16(p16, p16 + 3072, rgb_width, packed), one launch less).
 * gate (optional, gate.hip's int32 {signals, waits, ticket}; NULL: none): a signal added as the
 * dense-level launch starts (round 4: the side stream's next march starts beside the scatter
 * without a signal kernel of its own).
 * Replaces tcnn's hash-grid backward + apex FusedAdam's step over the whole model (train.py:136). */
int mfnerf_grid_encode_bw_binned_adam_all(const float* x, int64_t n, const int32_t* n_dev, float x_min, float x_range,
                                          const mfnerf_grid_desc* desc, const float* dL_dout, float* grads,
                                          int64_t n_params, void* workspace, int64_t n_slots, float* level_l1,
                                          const mfnerf_adam_fused* adam, int32_t* step_dev, mfnerf_amp_state* amp,
                                          void* packed, int rgb_width, int32_t* gate, mfnerf_stream_t stream);

/* out[l] += sum over rows i < n (or *n_dev) of |dL_dout[i][2l]| + |dL_dout[i][2l+1]| (f32). */
int mfnerf_grid_level_l1(const float* dL_dout, int64_t n, const int32_t* n_dev, int n_levels, float* out,
                         mfnerf_stream_t stream);


/* ---------------------------------------------------------------- NGP field head (MFMA) */

/* Weight blob for the two FullyFusedMLPs of NGP (networks.py:50-79) in this library's MFMA
 * fragment order (f16).  Built from fp32 tcnn-layout params by mfnerf_field_pack_weights. */
int64_t mfnerf_field_packed_bytes(int rgb_width);

/* params_xyz: (64*32 + 16*64) f32, row-major [out][in] per layer (tcnn layout, bias-free);
 * params_rgb: (W*32 + W*W + 16*W) f32.  Writes packed (mfnerf_field_packed_bytes). */
int mfnerf_field_pack_weights(const float* params_xyz, const float* params_rgb, int rgb_width, void* packed,
                              mfnerf_stream_t stream);

/* The same blob from the fp16 compute copy of the params (what packing the fp32 master gives). */
/* tcnn SphericalHarmonics degree 4 (networks.py:60-67 dir_encoder; input (d/|d| + 1)/2 as
 * networks.py:145-146 passes it): dirs01 (n, 3) f32 -> out (n, 16) f16.  The fused field head
 * computes the same encoding inside mfnerf_field_fw/bw; this is the tinycudann module route's. */
int mfnerf_sh4_fw(const float* dirs01, int64_t n, void* out_f16, mfnerf_stream_t stream);
int mfnerf_field_pack_weights_f16(const void* params_xyz_f16, const void* params_rgb_f16, int rgb_width, void* packed,
                                  mfnerf_stream_t stream);

/* NGP.forward (networks.py:134-155) on encoded features:
 *   h = xyz_mlp(feat); sigma = exp(h[0]); rgb = sigmoid(rgb_mlp([SH4((d/|d|+1)/2), h])).
 * feat: feat_plane_stride == 0 -> (n,32) f16 row-major (tcnn layout, mfnerf_grid_encode_fw);
 *       > 0 -> (16, feat_plane_stride) half2 level planes (mfnerf_grid_encode_fw_planar).
 * dirs (n,3) f32 (ignored when density_only) -> sigma (n) f32, rgb (n,3) f32. */
int mfnerf_field_fw(const void* feat_f16, int64_t feat_plane_stride, const float* dirs, int64_t n, const int32_t* n_dev, const void* packed,
                    int rgb_width, int density_only, float* sigma, float* rgb, mfnerf_stream_t stream);
/* The occupancy refresh's density query (networks.py:252-259, `density_grid_tmp[c, indices] =
 * self.density(xyzs)`): mfnerf_field_fw density_only over min(n, *n_dev) points, each sigma also
 * written to tmp[cell_idx[i]] (skipped for cell_idx < 0) -- the update's scatter in the same launch
 * (then call mfnerf_occupancy_update_dev with n_points = 0).  Duplicate cells: unordered, like
 * the reference's index_put; the engine's probes are distinct (mfnerf_occupancy_cells_unique). */
int mfnerf_field_fw_density_scatter(const void* feat_f16, int64_t feat_plane_stride, int64_t n, const int32_t* n_dev,
                                    const void* packed, int rgb_width, float* sigma, const int32_t* cell_idx,
                                    float* tmp, mfnerf_stream_t stream);

/* Backward of mfnerf_field_fw (recomputes the forward; same feat layouts).  dL_dsigma (n), dL_drgb (n,3) f32 ->
 * dL_dfeat (n,32) f32, and ADDS the weight grads into grad_xyz / grad_rgb (tcnn layout f32).
 * grad_scale: the loss scale -- factor applied to the incoming grads before the fp16 MFMA products
 * and removed from every output (keeps O(1e-6) per-sample grads out of the fp16 subnormals).
 * grad_scale == 0: the dynamic scale amp->scale, read on the device (amp required).
 * workspace: mfnerf_field_bw_workspace() bytes (per-workgroup weight-grad slab).
 * amp (optional): amp->nonfinite is set to 1 when any dL_dfeat or weight gradient is inf/nan (the
 * table gradient of mfnerf_grid_encode_bw is a weighted sum of dL_dfeat, so this flags the whole
 * step's gradient without scanning it; feeds mfnerf_adam_step's skip).
 * level_l1 (optional device f32[16], ACCUMULATED): the per-level L1 norm of dL_dfeat, i.e. what
 * mfnerf_grid_level_l1 computes, for free (the fixed-point scales of mfnerf_grid_encode_bw). */
int64_t mfnerf_field_bw_workspace(int64_t n, int rgb_width);
/* The weight-gradient slab rows field_bw writes into its workspace for rgb_width (the per-workgroup
 * partials mfnerf_field_bw_reduce folds); -1 for an unsupported width. */
int mfnerf_field_bw_slab_rows(int rgb_width);
int mfnerf_field_bw(const void* feat_f16, int64_t feat_plane_stride, const float* dirs, int64_t n, const int32_t* n_dev, const void* packed,
                    int rgb_width, const float* dL_dsigma, const float* dL_drgb, float grad_scale, float* dL_dfeat,
                    float* grad_xyz, float* grad_rgb, void* workspace, mfnerf_amp_state* amp, float* level_l1,
                    mfnerf_stream_t stream);

/* grad_xyz = grad_rgb = NULL in mfnerf_field_bw defers the weight-gradient fold: the per-block
 * partial sums stay in workspace (dL_dfeat, level_l1 and the data-gradient part of the non-finite
 * flag are complete when field_bw returns) and this call adds them into grad_xyz / grad_rgb in the
 * same fixed order (bit-identical to the undeferred call), raising nonfinite on an inf/nan weight
 * gradient.  The training step runs it on a second stream beside the table-gradient scatter, which
 * needs only dL_dfeat.  Part of the tcnn backward (networks.py:96-126) split for scheduling. */
int mfnerf_field_bw_reduce(int rgb_width, const void* workspace, float* grad_xyz, float* grad_rgb,
                           int32_t* nonfinite, mfnerf_stream_t stream);
/* mfnerf_field_bw_reduce STORING the folded sums (grad = fold, same order and bits) instead of adding
 * them: a gradient that holds only this step's weight gradient needs no zeroing first (the
 * data-parallel step, where nothing else adds into the MLPs' gradient). */
int mfnerf_field_bw_reduce_store(int rgb_width, const void* workspace, float* grad_xyz, float* grad_rgb,
                                 int32_t* nonfinite, mfnerf_stream_t stream);

/* ---------------------------------------------------------------- standalone FullyFusedMLP (MFMA)
 * tinycudann.Network / NetworkWithInputEncoding's network as MF-NeRF configures them one module at a
 * time (models/networks.py:36-79, tcnn FullyFusedMLP: bias-free, ReLU, output activation None or
 * Sigmoid, fp16): what the reference's own networks.py runs when tinycudann is this library
 * (module swap).  n_in = 32, width 64 or 128, n_hidden_layers 1 or 2, n_out <= 16
 * (padded to 16 as tcnn does).  params: tcnn layout, row-major [out][in] per layer, f32. */
int64_t mfnerf_mlp_n_params(int n_in, int width, int n_hidden, int n_out);
int64_t mfnerf_mlp_packed_bytes(int n_in, int width, int n_hidden, int n_out);
int mfnerf_mlp_pack(const float* params, int n_in, int width, int n_hidden, int n_out, void* packed,
                    mfnerf_stream_t stream);
/* x (n, 32) f16 -> out (n, 16) f16 (columns >= n_out hold the padded outputs). */
int mfnerf_mlp_fw(const void* x_f16, int64_t n, const void* packed, int n_in, int width, int n_hidden, int n_out,
                  int output_sigmoid, void* out_f16, mfnerf_stream_t stream);
/* dout (n, 16) f16 (zero beyond n_out) -> dx (n, 32) f32 (written), grad (n_params f32, ADDED:
 * dW = dZ^T A summed over samples in a fixed chunk order).  workspace: mfnerf_mlp_bw_workspace bytes. */
int64_t mfnerf_mlp_bw_workspace(int64_t n, int n_in, int width, int n_hidden, int n_out);
int mfnerf_mlp_bw(const void* x_f16, int64_t n, const void* packed, int n_in, int width, int n_hidden, int n_out,
                  int output_sigmoid, const void* dout_f16, float* dx, float* grad, void* workspace,
                  mfnerf_stream_t stream);


/* ---------------------------------------------------------------- occupancy grid refresh */

/* Device-only NGP.update_density_grid (networks.py:157-271, called every 16 steps by
 * train.py:165-168).  Three calls per refresh:
 *   1. mfnerf_occupancy_cells: the cells to probe, as jittered world points.  warmup != 0: every
 *      cell of every cascade (get_all_cells, networks.py:157-166); else per cascade n_uniform
 *      uniform cells + n_uniform cells drawn uniformly among {density_grid > density_threshold}
 *      (sample_uniform_and_occupied_cells, networks.py:168-192; the occupied list is in
 *      ascending morton order like torch.nonzero, and an empty set yields cell_idx -1).
 *      Outputs xyzs (n,3) f32 and cell_idx (n) i32 = cascade*G^3 + morton, with
 *      n = mfnerf_occupancy_points(...).  Random draws: counter-based hash of (seed, call_index).
 *   2. the caller evaluates sigma at xyzs (mfnerf_grid_encode_fw + mfnerf_field_fw density_only).
 *   3. mfnerf_occupancy_update: tmp = 0; tmp[cell_idx] = sigmas; density_grid = where(grid < 0,
 *      grid, max(grid*decay, tmp)) (decay = clamp(decay^(1/count_grid), 0.1, 0.95) when count_grid
 *      is given: erode); thr = min(mean(grid[grid > 0]), density_threshold) (NaN when no cell is
 *      positive, as Python's min(nan, x)); packbits(grid, thr) into bitfield.
 * tmp: cascades*G^3 f32 scratch.  workspace: mfnerf_occupancy_workspace() bytes, shared by 1 and 3. */
int64_t mfnerf_occupancy_workspace(int cascades, int grid_size);
int64_t mfnerf_occupancy_points(int cascades, int grid_size, int64_t n_uniform, int warmup);
int mfnerf_occupancy_cells(const float* density_grid, int cascades, int grid_size, float scale, int64_t n_uniform,
                           int warmup, float density_threshold, uint64_t seed, uint64_t call_index, float* xyzs,
                           int32_t* cell_idx, void* workspace, mfnerf_stream_t stream);
/* mfnerf_occupancy_cells with the call index read from (and then advanced in) device memory, so a
 * captured refresh draws new cells on every replay: call_index_dev (uint64, device) = the value
 * mfnerf_occupancy_cells' call_index would have; the same draws for the same index. */
int mfnerf_occupancy_cells_dev(const float* density_grid, int cascades, int grid_size, float scale, int64_t n_uniform,
                               int warmup, float density_threshold, uint64_t seed, uint64_t* call_index_dev,
                               float* xyzs, int32_t* cell_idx, void* workspace, mfnerf_stream_t stream);
int mfnerf_occupancy_update(float* density_grid, const float* sigmas, const int32_t* cell_idx, int64_t n_points,
                            int cascades, int grid_size, float decay, const float* count_grid, float density_threshold,
                            float* tmp, uint8_t* bitfield, void* workspace, mfnerf_stream_t stream);
/* The same probe de-duplicated (what the engine's refresh runs): of all the draws above only one
 * sigma per cell can reach the grid (`density_grid_tmp[c, indices] = ...`, networks.py:259, an
 * index_put whose duplicate writes land in no defined order), so the draws only mark their cells and
 * ONE jittered point is produced per distinct drawn cell -- keyed by (seed, call, cell) -- in ascending
 * row-major cell order within a cascade (x fastest; cell_idx still holds the cascade * G^3 + morton
 * index; the warm-up's every cell: morton order); *count_dev receives their number (<= the capacity
 * mfnerf_occupancy_points_unique(...)).  The set of probed cells is exactly the set the plain call
 * with the same seed and call index draws.  Deterministic.  The workspace must be zero-filled before
 * its first use (the call leaves its byte map zeroed); cascades*G^3 must be a multiple of 16.
 * mfnerf_occupancy_update_dev: mfnerf_occupancy_update over the first min(n_points, *n_dev) points;
 * tmp_zero = 1 promises tmp is all-zero on entry and leaves it zero (no fill launch). */
int64_t mfnerf_occupancy_points_unique(int cascades, int grid_size, int64_t n_uniform, int warmup);
int mfnerf_occupancy_cells_unique(const float* density_grid, int cascades, int grid_size, float scale,
                                  int64_t n_uniform, int warmup, float density_threshold, uint64_t seed,
                                  uint64_t call_index, float* xyzs, int32_t* cell_idx, int32_t* count_dev,
                                  void* workspace, mfnerf_stream_t stream);
int mfnerf_occupancy_cells_unique_dev(const float* density_grid, int cascades, int grid_size, float scale,
                                      int64_t n_uniform, int warmup, float density_threshold, uint64_t seed,
                                      uint64_t* call_index_dev, float* xyzs, int32_t* cell_idx, int32_t* count_dev,
                                      void* workspace, mfnerf_stream_t stream);
int mfnerf_occupancy_update_dev(float* density_grid, const float* sigmas, const int32_t* cell_idx, int64_t n_points,
                                const int32_t* n_dev, int cascades, int grid_size, float decay, const float* count_grid,
                                float density_threshold, float* tmp, int tmp_zero, uint8_t* bitfield,
                                void* workspace, mfnerf_stream_t stream);

/* ---------------------------------------------------------------- training batch */

/* One training batch from GPU-resident images (datasets/base.py:22-35 + train.py:93-105 get_rays,
 * datasets/ray_utils.py:50-70): per ray an image index (uniform over n_img; with same_image one
 * index for the whole batch) and a pixel index (uniform over hw), then
 *   rays_o = c2w[:, 3], rays_d = directions[pix] @ c2w[:, :3]^T, rgb = images[img, pix].
 * images (n_img, hw, 3) f32, poses (n_img, 3, 4) f32, directions (hw, 3) f32 (camera frame).
 * out (3, n_rays, 3) f32 = [rays_o | rays_d | rgb]; img_idx / pix_idx (n_rays) i32 optional.
 * Draws: counter-based hash of (seed, call[0], ray); call (optional device u64[2], zero-initialised)
 * is call[0] = the draw counter, incremented by the launch (by its last workgroup, call[1] being the
 * arrival ticket, 0 between launches), so graph replays sample fresh batches. */
int mfnerf_sample_rays(const float* images, const float* poses, const float* directions, int64_t n_img, int64_t hw,
                       int64_t n_rays, int same_image, uint64_t seed, uint64_t* call, float* out, int32_t* img_idx,
                       int32_t* pix_idx, mfnerf_stream_t stream);

/* mfnerf_sample_rays (no index outputs) fused with the ray-march prologue of the engine's step:
 * hits_t (n_rays,2) = ray_aabb_intersect of each drawn ray with the one box (center, half_size),
 * max_hits 1 (intersection.cu:5-56), with the near clamp t1 in [0, near) -> near
 * (rendering.py:29), and noise (n_rays) ~ U[0,1) (custom_functions.py:83) from the same counter
 * hash as the draws.  One launch instead of sample + AABB + clamp + noise kernels. */
int mfnerf_sample_rays_prep(const float* images, const float* poses, const float* directions, int64_t n_img,
                            int64_t hw, int64_t n_rays, int same_image, uint64_t seed, uint64_t* call, float* out,
                            const float* center, const float* half_size, float near, float* hits_t, float* noise,
                            mfnerf_stream_t stream);

/* ---------------------------------------------------------------- optimizer */

/* Adam (apex FusedAdam semantics, adam_w_mode=False, no weight decay; train.py:136):
 * m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2; p -= lr * (m/(1-b1^t)) / (sqrt(v/(1-b2^t)) + eps).
 * g is read as grad*grad_scale.  Optionally mirrors p into p_f16 (the fp16 compute copy).
 * step_dev (optional device i32): the number of completed steps; the update uses t = *step_dev+1
 * and the call then increments it (graph-replay safe).  Without step_dev, t = step.
 * lr_dev (optional device f32): learning rate read on the device (a schedule that does not
 * re-capture the graph); lr is used when it is NULL.
 * amp (optional): when amp->nonfinite != 0 the call changes nothing (params, m, v, p_f16 and
 * step_dev untouched) and increments amp->skipped -- torch GradScaler's skipped step on a
 * non-finite gradient (PL precision=16, train.py:287); amp->nonfinite is raised by
 * mfnerf_field_bw or mfnerf_check_finite.  Then GradScaler.update() (dynamic mode: backoff on a
 * skip, growth after growth_interval clean steps) and amp->nonfinite cleared -- done by the pass's
 * last workgroup (amp->ticket), no extra launch.
 * zero_grads != 0: grads is zeroed by the same pass (also on a skipped step), ready for the next
 * step's accumulation. */
int mfnerf_adam_step(float* params, float* grads, float* m, float* v, void* p_f16, int64_t n, float lr,
                     float beta1, float beta2, float eps, float grad_scale, int step, int32_t* step_dev,
                     const float* lr_dev, mfnerf_amp_state* amp, int zero_grads, mfnerf_stream_t stream);
/* The sharded update after the reduce-scatter (data parallel, train.py:277-287 DDP + apex
 * FusedAdam): mfnerf_flag_from_shard + mfnerf_adam_step(zero_grads = 0) in one launch.  The
 * non-finite flag is read from g_shard[0] (mfnerf_flag_to_shards put NaN there on any rank that
 * raised it; the reduction carries it to every shard); the last workgroup stores it in
 * amp->nonfinite for the bookkeeping, then zeroes zero[0, nz) (a per-step accumulator, e.g. the
 * grid's level L1 bounds).  amp and step_dev are required; g_shard is not modified. */
int mfnerf_adam_step_shard(float* params, const float* g_shard, float* m, float* v, void* p_f16, int64_t n, float lr,
                           float beta1, float beta2, float eps, float grad_scale, int32_t* step_dev, const float* lr_dev,
                           mfnerf_amp_state* amp, float* zero, int nz, mfnerf_stream_t stream);

/* mfnerf_grid_encode_bw_finish + mfnerf_adam_step (zero_grads on) in one pass, for a step with no
 * gradient exchange between them: grads[0, table_offset) are float gradients, grads[table_offset, ...)
 * the int32 fixed-point table sums mfnerf_grid_encode_bw_scatter left (level_l1 non-NULL there), the
 * dense prefix's in workspace's private copies.  Each value is converted exactly as the finish call
 * converts it and updated exactly as mfnerf_adam_step updates it (step_dev required, grad_scale 1);
 * grads and the private copies are zeroed (also on a skipped step).  n and table_offset: multiples
 * of 4, the table inside [table_offset, n).  level_l1 is zeroed after use, ready for the next step's
 * mfnerf_field_bw accumulation.  Replaces the two calls (and one pass over the gradient)
 * the reference makes as tcnn's backward + apex FusedAdam (train.py:136). */
int mfnerf_adam_step_fixed(float* params, float* grads, float* m, float* v, void* p_f16, int64_t n,
                           int64_t table_offset, const mfnerf_grid_desc* desc, void* workspace,
                           float* level_l1, float lr, float beta1, float beta2, float eps,
                           int32_t* step_dev, const float* lr_dev, mfnerf_amp_state* amp, mfnerf_stream_t stream);

/* The collective-free step's optimizer split in two (mfnerf_grid_encode_bw_binned_adam +
 * mfnerf_adam_step_fixed_partial): the partitioned accumulate applies Adam to the partitioned
 * tables' parameters itself, from each entry's finished int32 sum, and never writes their gradient
 * words (a record slot's overflow, added into them by atomics, is folded in and zeroed there); the
 * remaining pass updates [0, fused_from) only (fused_ovf non-NULL).  Same arithmetic, same bits as
 * the unsplit pair. */

int mfnerf_adam_step_fixed_partial(float* params, float* grads, float* m, float* v, void* p_f16, int64_t n,
                                   int64_t table_offset, const mfnerf_grid_desc* desc, void* workspace,
                                   float* level_l1, float lr, float beta1, float beta2, float eps,
                                   int32_t* step_dev, const float* lr_dev, mfnerf_amp_state* amp, int64_t fused_from,
                                   const int32_t* fused_ovf, mfnerf_stream_t stream);
/* value index (within the table) where the partitioned tables start, or -1 (nothing partitioned) */
int64_t mfnerf_grid_binned_first_value(const mfnerf_grid_desc* desc);
/* Values of the dense prefix (the leading own-table dense levels whose backward adds into private
 * copies and whose finish overwrites the gradient).  When it equals
 * mfnerf_grid_binned_first_value, mfnerf_grid_encode_bw_binned_float overwrites every table value
 * (no zeroing before it). */
int64_t mfnerf_grid_dense_values(const mfnerf_grid_desc* desc);
/* byte offset of the slot-overflow word inside the binned workspace sized for n_slots */
int64_t mfnerf_grid_encode_bw_binned_flag_offset(const mfnerf_grid_desc* desc, int64_t n_slots);

/* status[0] (device i32) = 1 if any of x (n f32, 16-byte aligned) is inf/nan, else 0 (a full scan;
 * the training step gets the same flag from mfnerf_field_bw's nonfinite argument instead). */
int mfnerf_check_finite(const float* x, int64_t n, int32_t* status, mfnerf_stream_t stream);

/* Sharded data parallel (mfnerf.dp.sharded_update): the step's non-finite flag rides the gradient
 * reduce-scatter.  mfnerf_flag_to_shards: if flag[0], grads[r*shard_len] = NaN for r < world (call
 * before the reduce-scatter); mfnerf_flag_from_shard: flag[0] = !isfinite(g_shard[0]) (after it).
 * Every rank then skips or updates together, with no extra collective. */
int mfnerf_flag_to_shards(float* grads, int64_t world, int64_t shard_len, const int32_t* flag, mfnerf_stream_t stream);
int mfnerf_flag_from_shard(const float* g_shard, int32_t* flag, mfnerf_stream_t stream);

/* A soft gate between two streams' captured graphs (no reference counterpart: it replaces the host
 * event the reference's PyTorch loop never needed, train.py:129-150 running one stream).  gate =
 * device int32[4] {signals, waits, -, timeouts}, zeroed once.  mfnerf_gate_signal adds a signal;
 * mfnerf_gate_wait (one thread) waits for the signal matching its own ticket, at most timeout_us,
 * then absorbs signals nobody waited for; a wait that gives up adds 1 to gate[3].
 * NO MEMORY ORDERING: signal and wait are relaxed atomics (an agent-scope release / acquire would
 * write back / invalidate the XCD's L2 on every poll), so the gate hands over no data -- a consumer
 * may not read anything the signaller wrote.  Ordering only: data hazards must be covered by stream
 * events, as the engine's are. */
int mfnerf_gate_signal(int32_t* gate, mfnerf_stream_t stream);
int mfnerf_gate_wait(int32_t* gate, int64_t timeout_us, mfnerf_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* MFNERF_H */
