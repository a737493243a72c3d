/*
 * rwrt.h -- C ABI of the MI355X batched Rossby-wave ray integrator.
 *
 * The reference (yinan-codes/Rossby-wave-ray-tracing) has no FFI: its ray loop
 * is selected by Python method dispatch, WR.ray_run -> WR.core_ray_run
 * ('numpy_rk45') -> WR.core_ray_run_rk45 (wr.py:889-911, 767-887).  The
 * entry points below are what that dispatch binds instead (ctypes, see
 * INTEGRATION.md); each cites the reference function it replaces.
 *
 * Conventions
 *  - Every pointer named d_* is DEVICE memory owned by the caller (the Python
 *    host keeps it in PyTorch-ROCm tensors).  The library never allocates or
 *    frees caller memory.
 *  - All calls are asynchronous and ordered on `stream` (a hipStream_t; NULL =
 *    the default stream).  Status codes report argument and launch errors;
 *    per-ray failure is data (NaN), exactly as in the reference.
 *  - fp64 throughout; the fields are the reference's 18-field stack.
 *  - The ray-loop entry points (rwrt_rk45_run, rwrt_rk45_run_tv, rwrt_rk4_run)
 *    take an execution context, rwrt_ctx, that owns the library's own scratch
 *    (a per-ray frozen flag, a side stream and its events).  Nothing else in
 *    the library holds state between calls: calls through DISTINCT contexts
 *    are reentrant and may run concurrently on different streams or threads.
 *    One context may be shared by threads (its calls are serialised on the
 *    host) and used on several streams (a call waits on the device for the
 *    context's previous call before reusing its scratch).
 */
#ifndef RWRT_H
#define RWRT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RWRT_ABI_VERSION 4  /* 3: constant row tails (rwrt_rk45_run_tails, rwrt_expand_tails);
                               4: row blocks for the live rays only (rwrt_rk45_run_slots) */
#define RWRT_NFIELD_REF 18  /* BS.fields[..., 18]            (bs.py:349-368) */
#define RWRT_NFIELD_PACK 12 /* 11 hot fields + 1 pad per grid point           */
#define RWRT_NVAR 5         /* y = (lon, lat, k, l, amp)     (wr.py:768-776)  */
#define RWRT_NMERC 12       /* fmu .. fmqyy                  (bs.py:885-887)  */
#define RWRT_NOUT 8         /* per output row: lon lat k l amp ug vg nacc     */
#define RWRT_NSTATE 12      /* per ray: y[5] f[5] t h_abs                     */

typedef enum {
  RWRT_OK = 0,
  RWRT_ERR_ARG = 1,        /* bad argument (message in rwrt_last_error)     */
  RWRT_ERR_HIP = 2,        /* HIP launch / runtime error                     */
  RWRT_SOLVER_FAILED = 3   /* rkf45.py:423-425 "All nan" (set by the host)   */
} rwrt_status;

/* Grid of BS.fields: W = nlon (+1 cyclic pad column, bs.py:370-372) columns,
 * H = nlat rows.  lon0/dlon, lat0/dlat are bs.lon[0], bs.lon[1]-bs.lon[0],
 * bs.lat[0], bs.lat[1]-bs.lat[0] of the float32-rounded grid
 * (bs.py:225-236, interpolation.py:78-82). */
typedef struct {
  int32_t ncol;
  int32_t nrow;
  double lon0, dlon;
  double lat0, dlat;
} rwrt_grid;

/* Solver parameters of WR.core_ray_run_rk45 / RK45 (wr.py:792-794). */
typedef struct {
  double rtol;      /* max(rtol, 100 eps)          rkf45.py:21-26  */
  double atol;
  double min_step;  /* Global_Minstep              rkf45.py:362    */
  double cut_off;   /* jump mask threshold, rad    wr.py:170       */
  int32_t nt;       /* rows of the history         wr.py:157       */
  int32_t reserved;
  double tstep;     /* output interval = RK4 step  wr.py:147       */
} rwrt_params;

/* A time-varying basic state (this framework's extension for BASELINE
 * configs[4]; the reference's fun ignores t, wr.py:784-789): nlev packed
 * levels [nlev][ncol][nrow][12] (fp64, or fp32 when fp32 != 0; fp32 == 2
 * also computes the RHS in fp32 -- not the reference's arithmetic) valid at
 * t0 + j*dt seconds of ray time.  The RHS interpolates each level bilinearly
 * exactly like the static state and then linearly in time:
 * s = (t - t0)/dt, j = clip(floor(s), 0, nlev-2), w = clip(s - j, 0, 1),
 * field = f_j (1 - w) + f_{j+1} w. */
typedef struct {
  const void* d_levels;
  int32_t nlev;
  int32_t fp32;
  double t0;
  double dt;
} rwrt_background;
const char* rwrt_version(void);

/* Execution context of the ray-loop entry points: created
 * for one HIP device, destroyed when no call through it is pending (destroy
 * waits for the last call's kernels before freeing its scratch). */
typedef struct rwrt_ctx rwrt_ctx;
rwrt_status rwrt_ctx_create(int32_t device, rwrt_ctx** out);
rwrt_status rwrt_ctx_destroy(rwrt_ctx* ctx);
/* Rays per wavefront in the latency mode of rwrt_rk45_run (n_heavy > 0) on
 * this context: 1..16 (default 16 = 64 rays per CU).  Fewer rays per wave
 * make each heavy ray's attempts faster (its wave stalls less often on the
 * other rays' cell refills and interval ends) at more CUs per heavy ray.
 * Schedule only: results do not depend on it. */
rwrt_status rwrt_ctx_set_latency_density(rwrt_ctx* ctx, int32_t rays_per_wave);
/* Rays per wavefront of this context's fp64 time-varying ray loops
 * (rwrt_rk45_run_tv*, levels with fp32 == 0): 64 (default; the lower
 * bracketing level cached per lane in LDS, the upper one gathered) or 32
 * (lane pairs: lanes L and L + 32 run the same ray, each caching and blending
 * one bracketing level, exchanged by v_permlane32_swap -- no HBM gathers
 * while a ray stays in its cell and level pair, half the LDS-DMA per refill;
 * RayEngine's default, C5 fp64 1.21 -> 1.61e9 with the other round-5 changes).
 * Schedule only: results do not depend on it (ABI 3). */
rwrt_status rwrt_ctx_set_tv_lanes(rwrt_ctx* ctx, int32_t lanes);
/* Drain-time hand-off of this context's static-state ray loops (ABI 4): once
 * a call's work queue is drained, a wavefront with at most max_rays rays left
 * (0 = off, at most 16; default 16) continues them four lanes per ray, in the
 * latency mode's layout, from exactly where they stopped (between two
 * attempts).  Schedule only: results do not depend on it.  A call's d_work[0]
 * counts the rays it handed off (diagnostic). */
rwrt_status rwrt_ctx_set_handoff(rwrt_ctx* ctx, int32_t max_rays);
/* Diagnostic ray trace of the context's rwrt_rk45_run calls (NULL / 0: off):
 * for queue positions w < capacity of the order, the ray's lane records
 * d_trace[w * 10 + 0..9] = {ray, hardware id (HW_REG_HW_ID: wave, SIMD, CU,
 * SE fields), XCC id, start and end of the ray's integration in the launch
 * (s_memrealtime, 100 MHz), attempts made, 1 if in latency mode else 0,
 * block index, start and end in shader clocks (s_memtime)} -- where, how long
 * and at what clock the heaviest rays run (the makespan of a launch is
 * theirs).  Costs one compare per ray when off. */
rwrt_status rwrt_ctx_set_trace(rwrt_ctx* ctx, int64_t* d_trace, int64_t capacity);
/* Last error message of the calling thread ("" if none). */
const char* rwrt_last_error(void);

/* Device layout of BS.fields (bs.py:349-372): d_fields is the reference stack
 * [ncol][nrow][18] fp64; d_packed receives [ncol][nrow][12] (the 11 fields the
 * hot path reads -- u v ux uy vx vy qx qy qxx qxy qyy -- plus a zero pad). */
rwrt_status rwrt_pack_fields(const rwrt_grid* g, const double* d_fields,
                             double* d_packed, void* stream);

/* BS.cal_bs_mercator_point(lon, lat, mode='numpy') (bs.py:513-519,781-887):
 * d_out[12][n] = fmu fmv fmux fmuy fmvx fmvy fmqx fmqy fmqxx fmqxy fmqyx fmqyy. */
rwrt_status rwrt_mercator_point(const rwrt_grid* g, const double* d_packed,
                                int64_t n, const double* d_lon,
                                const double* d_lat, double* d_out,
                                void* stream);

/* WR.diffun_numpy(y)[0][0:5] (wr.py:492-556 with core_diffun wr.py:44-82 and
 * cal_ugvg 'extent' wn.py:266-294): d_y[5][n] -> d_dydt[5][n]. */
rwrt_status rwrt_rhs(const rwrt_grid* g, const double* d_packed, int64_t n,
                     const double* d_y, double* d_dydt, void* stream);

/* One Dormand-Prince 5(4) attempt: rk_step (rkf45.py:259-321) followed by
 * _estimate_error_norm (rkf45.py:368-373, scale rkf45.py:442-445).
 * d_y, d_f: [5][n]; d_h: [n] (signed step).  Outputs d_K[7][5][n],
 * d_ynew[5][n], d_err[n] (NaN kept, as the reference returns it). */
rwrt_status rwrt_dp54_attempt(const rwrt_grid* g, const double* d_packed,
                              int64_t n, const double* d_y, const double* d_f,
                              const double* d_h, double rtol, double atol,
                              double* d_K, double* d_ynew, double* d_err,
                              void* stream);

/* Initial rays WR.ray_initial_numpy (wr.py:344-395) on the device, per
 * (source, zonal wavenumber): the Mercator point at the source
 * (cal_bs_mercator_point, bs.py:781-887), the meridional wavenumbers of the
 * t = 0 dispersion relation (cal_ky_numpy, bs.py:985-1040 -- np.roots
 * restated operation for operation: companion matrix, LAPACK zgeev's
 * zgebal + zlahqr, csrc/nproots.h), change_roots_order (bs.py:942-982) and
 * the t = 0 group velocity (cal_ugvg_numpy, wn.py:209-259).
 *  d_src_lon, d_src_lat, d_src_cos [nsource]: source position (radians, as
 *    set_source_matrix makes it, wr.py:236-258) and np.cos(lat) from the
 *    host libm -- the one transcendental of this path, so that it is the
 *    reference's own value.
 *  d_zwn[4][nzwn] = {k, k**2, k**3, freq / k * R} as NumPy evaluates them
 *    (bs.py:1005-1012).
 *  d_rows[7][3][nsource][nzwn] = lon lat k l amp ug vg (wr.py:160-167
 *    layout of row 0; NaN where a slot has no real root).
 *  d_info[1] (int32, zeroed by this call) counts polynomials with
 *    non-finite coefficients -- np.linalg.eigvals raises LinAlgError there;
 *    the host raises too when it is non-zero. */
rwrt_status rwrt_ray_initial(const rwrt_grid* g, const double* d_packed,
                             int64_t nsource, const double* d_src_lon,
                             const double* d_src_lat, const double* d_src_cos,
                             int32_t nzwn, const double* d_zwn, double* d_rows,
                             int32_t* d_info, void* stream);
/* Solver construction: RungeKutta.__init__ (rkf45.py:335-366) with
 * select_initial_step (rkf45.py:34-99) on d_y0[5][nray].
 * Writes d_state[12][nray] = y f t(=0) h_abs, zeroes d_count[nray][2]
 * (accepted, rejected), sets d_nanrow[nray] = nt and d_live[nray] (1 if the
 * ray's state has a finite mean, rkf45.py:400-403).  d_summary[2] (int64,
 * zeroed here) accumulates {live rays, live rays with a finite h_abs}: the
 * host raises RWRT_SOLVER_FAILED when the first is > 0 and the second is 0
 * (the only way rkf45.py:423-425 can trigger). */
rwrt_status rwrt_rk45_init(const rwrt_grid* g, const double* d_packed,
                           int64_t nray, const double* d_y0,
                           const rwrt_params* p, double* d_state,
                           int64_t* d_count, int32_t* d_nanrow,
                           int32_t* d_live, int64_t* d_summary, void* stream);

/* The ray loop WR.core_ray_run_rk45 (wr.py:767-887) for output rows
 * it_begin <= i < it_end (1 <= it_begin < it_end <= nt): every ray is stepped
 * to d_tbound[i] (t_eval, wr.py:798-801) with the reference's step control
 * (rkf45.py:222-253,375-514), then masked (wr.py:838-850) and its group
 * velocity recomputed (wr.py:856-865).  Rays are taken from device work
 * queues in the order d_order[nray] (NULL = 0..nray-1); the first n_heavy
 * entries (live rays, at most 4 x rays-per-wave per CU on half the CUs) run
 * in latency mode -- four lanes of a wave per ray, in the first blocks of the
 * same grid (pass the rays expected to be slowest; 0 = none).
 * Output row r of
 * ray j is d_out[(j*(it_end-it_begin) + r)*8 + {lon,lat,k,l,amp,ug,vg,nacc}].
 * d_state / d_count / d_nanrow carry the per-ray solver state across calls
 * (time chunking).  d_work: >= 2 int32 of scratch (queue heads), reset by
 * this call on `stream`.  Results do not depend on the order or n_heavy.
 * Rays frozen at the call's start (NaN in their state) are flagged in the
 * context's scratch (1 byte per ray, grown on demand) and their rows written
 * by a kernel on the context's side stream; `stream` waits for it, so the
 * call remains one stream-ordered operation (also for rwrt_rk45_run_tv and
 * rwrt_rk4_run). */
rwrt_status rwrt_rk45_run(rwrt_ctx* ctx, const rwrt_grid* g, const double* d_packed,
                          int64_t nray, const rwrt_params* p,
                          const double* d_tbound, int32_t it_begin,
                          int32_t it_end, const int64_t* d_order,
                          int64_t n_heavy, double* d_state, int64_t* d_count,
                          int32_t* d_nanrow, double* d_out, int32_t* d_work,
                          void* stream);

/* rwrt_rk45_run with constant row tails (ABI 3).  A ray frozen at the call's
 * start (a NaN in its state, rkf45.py:400-403: dead root slots, rays masked
 * by wr.py:838-850 in an earlier call) repeats one row for the whole call
 * (wr.py:868-876 stores the unchanged state).  Instead of writing that row
 * into d_out for every row, the call stores it once:
 *  d_tail_from[nray] (int32): the first row i (it_begin <= i <= it_end) from
 *    which ray j's rows of this call all equal d_tail_row[j] and are NOT
 *    written to d_out; it_end when the ray has no constant tail (every row of
 *    it is in d_out).  This build gives the rays frozen at the call's start
 *    it_begin and every other ray it_end (a ray that freezes during the call
 *    writes its remaining rows, as rwrt_rk45_run does).
 *  d_tail_row[nray][8] (16-byte aligned): the tail row of ray j (meaningful
 *    where d_tail_from[j] < it_end).
 * rwrt_expand_tails writes the tails into d_out for a consumer that wants the
 * rows dense: then d_out equals rwrt_rk45_run's bit for bit, as do the state,
 * counters and nanrow after every call.  NULL d_tail_from and d_tail_row:
 * rwrt_rk45_run itself.  (C3: 116 GB of constant rows per 90-day step that
 * are never written.) */
rwrt_status rwrt_rk45_run_tails(rwrt_ctx* ctx, const rwrt_grid* g, const double* d_packed,
                                int64_t nray, const rwrt_params* p,
                                const double* d_tbound, int32_t it_begin,
                                int32_t it_end, const int64_t* d_order,
                                int64_t n_heavy, double* d_state, int64_t* d_count,
                                int32_t* d_nanrow, double* d_out, int32_t* d_tail_from,
                                double* d_tail_row, int32_t* d_work, void* stream);
/* d_out[(j*(it_end-it_begin) + r)*8 + 0..7] := d_tail_row[j][0..7] for every
 * ray j and row it_begin + r >= d_tail_from[j] (the dense rows of a tails
 * call); other rows are not touched. */
rwrt_status rwrt_expand_tails(int64_t nray, int32_t it_begin, int32_t it_end,
                              const int32_t* d_tail_from, const double* d_tail_row,
                              double* d_out, void* stream);

/* ABI 4: rows only for the rays live at the call's start.  rwrt_row_slots
 * numbers the rays whose state has a finite mean (rkf45.py:400-403: the rays
 * a call steps; every other ray repeats one row, its tail) in ray order:
 *  d_row_slot[nray] (int32) := j's index among them, -1 for a frozen ray;
 *  d_nslot[0] (int64) := their number.
 * rwrt_rk45_run_slots is rwrt_rk45_run_tails with ray j's rows at
 * d_out[(d_row_slot[j]*(it_end-it_begin) + r)*8 + 0..7]: d_out holds
 * nslot x rows x 8 doubles instead of nray x rows x 8 (C3: the 716 400 live
 * rays of 2.40 M slots, 49.5 GB instead of 166 GB for a 1 080-row call).
 * d_row_slot must come from rwrt_row_slots on the call's own d_state (after
 * the previous call); tails are required.  rwrt_expand_slots writes the dense
 * rows d_out[nray][rows][8] of such a call from its row blocks d_rows and its
 * tails: equal bit for bit to rwrt_rk45_run's d_out. */
rwrt_status rwrt_row_slots(int64_t nray, const double* d_state, int32_t* d_row_slot, int64_t* d_nslot,
                           void* stream);
rwrt_status rwrt_rk45_run_slots(rwrt_ctx* ctx, const rwrt_grid* g, const double* d_packed,
                                int64_t nray, const rwrt_params* p,
                                const double* d_tbound, int32_t it_begin,
                                int32_t it_end, const int64_t* d_order,
                                int64_t n_heavy, double* d_state, int64_t* d_count,
                                int32_t* d_nanrow, double* d_out, const int32_t* d_row_slot,
                                int32_t* d_tail_from, double* d_tail_row, int32_t* d_work,
                                void* stream);
rwrt_status rwrt_expand_slots(int64_t nray, int32_t it_begin, int32_t it_end, const int32_t* d_row_slot,
                              const int32_t* d_tail_from, const double* d_tail_row, const double* d_rows,
                              double* d_out, void* stream);

/* Fixed-step RK4 ray loop, the reference's default integrator:
 * WR.core_ray_run_numpy (wr.py:702-765) with rk4_step_numpy (wr.py:583-622)
 * and core_rk4_step (wr.py:89-95), for rows it_begin <= i < it_end, dt =
 * p->tstep.  A ray whose stage input is masked (|lat| >= pi/2 or |l| >= 100)
 * keeps its state for that step.  d_state rows 0..4 hold y (set them to the
 * initial rows before the first call); d_count[nray][2] = {steps taken, steps
 * held} -- held by a masked stage 2-4, or by a masked first stage, which
 * holds the ray for every remaining step (the step of a state with a NaN in
 * lon/lat/k/l is counted in neither); d_nanrow / d_out / d_work as for
 * rwrt_rk45_run (nacc column = steps taken); rays with such a NaN at the
 * call's start are written from the context's side stream as in
 * rwrt_rk45_run. */
rwrt_status rwrt_rk4_run(rwrt_ctx* ctx, const rwrt_grid* g, const double* d_packed,
                         int64_t nray, const rwrt_params* p, int32_t it_begin,
                         int32_t it_end, const int64_t* d_order,
                         double* d_state, int64_t* d_count, int32_t* d_nanrow,
                         double* d_out, int32_t* d_work, void* stream);

/* BS.ready on the device (bs.py:264-279 vorticity, bs.py:121-200 finite
 * differences, bs.py:291-305 smth9, bs.py:318-372 the stack): writes the
 * packed record [nlon+1][nlat][12] of one basic state (fp64, or fp32 when
 * fp32 != 0) -- the 11 hot fields bit-identical to BS.fields.
 *  d_u, d_v [nlat][nlon] float32 as read from the file (ascending latitude;
 *    the host flips a descending file like bs.py:251-256).
 *  d_trig[3][nlat]: np.cos(lat) (for u cos(lat)), then np.cos and np.sin of
 *    lat[1:-1] at indices 1..nlat-2 (host libm, the reference's values).
 *  dx, dy: BS.dx, BS.dy (bs.py:77-78).  d_scratch: 4*nlon*nlat doubles. */
rwrt_status rwrt_bs_ready(int32_t nlon, int32_t nlat, const float* d_u,
                          const float* d_v, const double* d_trig, double dx,
                          double dy, double* d_scratch, void* d_packed,
                          int32_t fp32, void* stream);
/* rwrt_rk45_init / rwrt_rk45_run on a time-varying background (same state,
 * queue and output conventions).  Steps reuse K6 = fun(t + h, y_new) as the
 * next f (FSAL, scipy's RK45 convention); the per-row group velocity is
 * evaluated at the row time t_bound. */
rwrt_status rwrt_rk45_init_tv(const rwrt_grid* g, const rwrt_background* b,
                              int64_t nray, const double* d_y0,
                              const rwrt_params* p, double* d_state,
                              int64_t* d_count, int32_t* d_nanrow,
                              int32_t* d_live, int64_t* d_summary, void* stream);
rwrt_status rwrt_rk45_run_tv(rwrt_ctx* ctx, const rwrt_grid* g, const rwrt_background* b,
                             int64_t nray, const rwrt_params* p,
                             const double* d_tbound, int32_t it_begin,
                             int32_t it_end, const int64_t* d_order,
                             int64_t n_heavy, double* d_state, int64_t* d_count,
                             int32_t* d_nanrow, double* d_out, int32_t* d_work,
                             void* stream);
/* n_heavy > 0 on a time-varying background (fp64 or fp32 levels; not with
 * fp32 arithmetic, fp32 == 2): the first n_heavy rays of d_order (at most 4
 * per CU on half the CUs) run one per wavefront, replicated on its 64 lanes,
 * their lookups served from an 8 x 8-point block of both bracketing levels in
 * the wave's LDS (reloaded by all 64 lanes at once) -- a schedule, results
 * are unchanged (ABI 3). */
/* rwrt_rk45_run_tv with constant row tails (as rwrt_rk45_run_tails). */
rwrt_status rwrt_rk45_run_tv_tails(rwrt_ctx* ctx, const rwrt_grid* g, const rwrt_background* b,
                                   int64_t nray, const rwrt_params* p,
                                   const double* d_tbound, int32_t it_begin,
                                   int32_t it_end, const int64_t* d_order,
                                   int64_t n_heavy, double* d_state, int64_t* d_count,
                                   int32_t* d_nanrow, double* d_out, int32_t* d_tail_from,
                                   double* d_tail_row, int32_t* d_work, void* stream);
/* rwrt_rk45_run_tv with row blocks for the live rays only (as rwrt_rk45_run_slots). */
rwrt_status rwrt_rk45_run_tv_slots(rwrt_ctx* ctx, const rwrt_grid* g, const rwrt_background* b,
                                   int64_t nray, const rwrt_params* p,
                                   const double* d_tbound, int32_t it_begin,
                                   int32_t it_end, const int64_t* d_order,
                                   int64_t n_heavy, double* d_state, int64_t* d_count,
                                   int32_t* d_nanrow, double* d_out, const int32_t* d_row_slot,
                                   int32_t* d_tail_from, double* d_tail_row, int32_t* d_work,
                                   void* stream);
/* The time-varying RHS at per-point times: d_t[n], d_y[5][n] -> d_dydt[5][n]. */
rwrt_status rwrt_rhs_tv(const rwrt_grid* g, const rwrt_background* b, int64_t n,
                        const double* d_t, const double* d_y, double* d_dydt,
                        void* stream);
/* Stepper known-answer tests: the same device stepper on the analytic ODEs of
 * the rkf45.py demos (rkf45.py:839-882), driven like rk45_simple_current
 * (rkf45.py:672-724).  kind: 0 dx/dt = 2t, 1 dx/dt = e^(0.1 t), 2 Lorenz
 * (nvar 1, 1, 3).  d_y0[nvar][ncol]; d_teval[nt]; d_out[ncol][nt][nvar]. */
rwrt_status rwrt_kat_rk45(int32_t kind, int64_t ncol, const double* d_y0,
                          int32_t nt, const double* d_teval, double rtol,
                          double atol, double min_step, double* d_out,
                          void* stream);

/* Device math self-test: d_out[i] = f(d_x[i], d_y[i]) with the exact device
 * routines the kernels use.  kind: 0 sin(x), 1 cos(x), 2 tan(x), 3 pow(x, y),
 * 4 atan2(x, y), 5 Python x % y (fmod-based), 6 sqrt(x), 7 x / y, 8 floor(x),
 * 9/10 sin/cos through sincos(x), 11 x / 6.3712e6 (the kernels' exact division
 * by the earth radius), 12 fmod(x, y) for y > 0 (the kernels' exact fmod),
 * 13 x % (2 pi) and 14 (x % (2 pi)) % (2 pi) as the kernels evaluate them,
 * 15 x / y by a shared reciprocal, 16 np.floor(x).astype(int32),
 * (17-22: retired device-libm restatements), 23/24 x / y through the interleaved
 * division pair (as its first / second quotient), 25/26/27/28 the reference
 * NumPy's sin/cos/tan/power as restated in csrc/np_math.h, 29 the restated
 * VRCP14PD, 30/31/32 sin/cos/tan and 33 pow exactly as the kernels evaluate
 * them, 34 x / y by the RHS's shared-reciprocal division (qdiv), 35 1.0
 * where that division is inside its exact range (DivGuard), else 0.0, and
 * 36/37 the jump mask's verdict (wr.py:844-850; 1.0: a jump) for a step of
 * (dlat, dlon) = (x, y) from (lon, lat) = (1.0, 0.6) rad at cut_off 0.05 rad,
 * 36 with the kernels' polynomial "no jump" shortcut, 37 without it.
 * Lets the tests prove which operations are bit-exact on the GPU (IEEE
 * division, sqrt, fmod) and measure the last-bit agreement of the rest. */
rwrt_status rwrt_selftest_math(int32_t kind, int64_t n, const double* d_x,
                               const double* d_y, double* d_out, void* stream);

/* HOST routine (no device call; the drop-in's delivery into the reference
 * arrays, wr.py:868-876): rows [0, nrows) of a host block dst[nrows][ncol]
 * (row stride ld doubles) become prev[ncol] -- the row before the block --
 * except the nsrc columns cols[] (strictly ascending, < ncol), which take
 * src[nrows][nsrc] (row stride ld_src).  A ray whose rows in a launch are all
 * bitwise equal to its previous row (a frozen ray: rkf45.py:400-403) is then
 * never shipped over PCIe; the block equals what a full copy would give, bit
 * for bit.  Reentrant (callers split the rows over threads). */
rwrt_status rwrt_host_fill_rows(double* dst, int64_t nrows, int64_t ncol, int64_t ld,
                                const double* prev, const double* src, int64_t nsrc,
                                int64_t ld_src, const int64_t* cols);

#ifdef __cplusplus
}
#endif

#endif /* RWRT_H */
