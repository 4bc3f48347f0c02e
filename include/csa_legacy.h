/*
 * csa_legacy.h -- C ABI of the MI355X-native LEGACY Monte Carlo engine
 * (libcsa_legacy.so, built from citizensassemblies-replication_amd/csrc/).
 *
 * The reference (sirandreww/citizensassemblies-replication) has no FFI: its
 * boundary is a Python call surface.  Each entry point below names the
 * reference function it replaces (file:line); the Python mirror in
 * citizensassemblies-replication_amd/{legacy,analysis}.py binds them through
 * ctypes and keeps the reference signatures.  INTEGRATION.md shows the
 * binding a maintainer adds to the reference.
 *
 * Conventions
 *   - plain C types only; the caller owns every buffer; no exception crosses
 *     the ABI; every function returns a CSA_* status code (0 = ok) and leaves
 *     a thread-local message in csa_last_error().
 *   - an instance lives on the HIP device that was current when it was
 *     created.  Multi-GPU: one process per GPU with the RCCL exchange in the
 *     Python layer (DESIGN.md "Multi-GPU"), or several devices of one process
 *     through csa_legacy_sample_devices (replicas owned by the handle).
 *   - agent ids are 0..n-1 = pool row order (analysis.py:131-133); feature
 *     ids are 0..F-1 in category-major CSV order (analysis.py:114-124).
 *   - randomness: Philox4x32-10 verification-mode stream, keyed by
 *     (seed, panel, attempt, step) -- see oracle/philox.py for the contract.
 *   - bitmask panels: uint64 words, W = ceil(n/64) per panel, agent p is
 *     bit (p & 63) of word (p >> 6).
 */
#ifndef CSA_LEGACY_H
#define CSA_LEGACY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes --------------------------------------------------------- */
#define CSA_OK 0
#define CSA_E_INVALID 1        /* bad argument / inconsistent instance                         */
#define CSA_E_BAD_QUOTAS 2     /* sum(min) <= k <= sum(max) violated: analysis.py:174-176 assert */
#define CSA_E_NO_CANDIDATE 3   /* no candidate feature: the reference's KeyError, legacy.py:188  */
#define CSA_E_ATTEMPT_LIMIT 4  /* new: the reference restarts forever (analysis.py:146)          */
#define CSA_E_UNSUPPORTED 5    /* instance exceeds the kernels' limits (F > 64, n > 16384, ...)  */
#define CSA_E_HIP 6            /* HIP runtime / device error                                     */
#define CSA_E_SELECTION 7      /* one attempt raised SelectionError (legacy.py:34-36)            */

/* ---- flags for csa_legacy_sample ----------------------------------------- */
#define CSA_WANT_PANELS 0x1u   /* copy packed panels (n_panels * W uint64) to panels_out   */
#define CSA_WANT_COUNTS 0x2u   /* per-person counts (analysis.py:179,187)                  */
#define CSA_WANT_PAIRS 0x4u    /* pair co-selection counts (PairHistogram, analysis.py:68) */
#define CSA_WANT_UNIQUE 0x8u   /* number of distinct panels (found_panels, analysis.py:171) */

typedef struct csa_instance csa_instance;

int csa_version(void);                 /* ABI version, currently 1 */
const char *csa_last_error(void);      /* thread-local message of the last failing call */
int csa_device_count(int32_t *out);    /* HIP devices visible to this process */
/* The calling thread's current HIP device (hipGetDevice).  An instance lives on the device that was
 * current at csa_instance_create; the stream-ordered entry points run on the caller's stream, so a
 * caller keeps one instance per device it launches on (the Python layer does: EncodedInstance.handle). */
int csa_current_device(int32_t *out);

/* Encode an instance (replaces read_instance's dicts, analysis.py:108-138).
 * person_feat: n*C global feature ids (row p = agent p, column c = category c);
 * fmin/fmax: F quotas; feat_cat: F category ids (features of one category are
 * contiguous, category-major).  Uploads the feature bitmasks to the current
 * device.  Initial state: selected = 0, remaining = pool counts, all present. */
int csa_instance_create(int32_t n, int32_t C, int32_t F, const int32_t *person_feat,
                        const int32_t *fmin, const int32_t *fmax, const int32_t *feat_cat,
                        csa_instance **out);
void csa_instance_destroy(csa_instance *inst);
/* n, C, F, W = ceil(n/64) */
int csa_instance_info(const csa_instance *inst, int32_t *n, int32_t *C, int32_t *F, int32_t *W);
/* Replace the initial draw state (for find_random_sample_legacy called on
 * partially used dicts): sel/rem: F counters ("selected"/"remaining" of
 * legacy.py's category items), present: W words of the people dict's keys.
 * Any NULL argument restores that part of the default state. */
int csa_instance_set_state(csa_instance *inst, const int32_t *sel, const int32_t *rem,
                           const uint64_t *present);

/* Draw statistics (SURVEY.md section 5 "Metrics"; the reference prints "Rejected" for every
 * min-quota rejection, analysis.py:159, and restarts silently on SelectionError, analysis.py:152-153).
 * Totals over every legacy_find-semantics draw launched on the instance -- csa_legacy_sample,
 * csa_legacy_sample_devices (its per-device replicas included), csa_legacy_find,
 * csa_first_panel_not_in, csa_draw_async / csa_draw_picks_async -- since creation or the last reset
 * (csa_legacy_attempt's single attempts are not counted):
 *   out[0] attempts = accepted panels + out[1] + out[2]
 *   out[1] SelectionError restarts (legacy.py:34-36 raised inside an attempt)
 *   out[2] min-quota rejections (check_min_cats false after k picks, legacy.py:160-168)
 * Synchronises the instance's device(s); reset != 0 zeroes the totals after reading them. */
int csa_instance_draw_stats(csa_instance *inst, int32_t reset, uint64_t *out);
/* Zero the draw statistics without a device-wide synchronisation: with a stream, a memset
 * ordered on it (draws the caller enqueues after it on that stream count from zero); with NULL,
 * after the instance's own streams (csa_legacy_sample's pipeline) are idle.  Other streams of the
 * device are never waited for. */
int csa_instance_draw_stats_reset(csa_instance *inst, void *stream);
/* The same totals as csa_instance_draw_stats (this instance only, not csa_legacy_sample_devices'
 * replicas) written to device memory d_out[0..2] by a kernel on `stream`: no host wait, so a
 * caller orders it after its draws and reads it together with its other results. */
int csa_instance_draw_stats_async(csa_instance *inst, uint64_t *d_out, void *stream);

/* check_same_address (legacy.py:78-99, 103-113): addr_next (n int32) links the agents that share
 * an address (the check_same_address_columns values) into rings, agent order: addr_next[p] = the
 * next agent at p's address, p itself when p lives alone.  With a ring set, every pick deletes
 * the remaining agents at its address (really_delete_person(selected=False)) before the
 * full-category cascades; all draws of the instance then run draw_kernel<64, ..., true>.
 * NULL removes the rings (the default: the reference harness passes False, analysis.py:150). */
int csa_instance_set_address(csa_instance *inst, const int32_t *addr_next);

/* ---- host-buffer API (blocking) ------------------------------------------ */

/* legacy_probabilities (analysis.py:162-191) for panels
 * [panel_begin, panel_begin + n_panels): draw every panel with restarts
 * (legacy_find, analysis.py:141-159), then reduce.  Outputs (host memory,
 * each may be NULL when its flag is clear):
 *   panels_out    n_panels * W uint64, panel order            (CSA_WANT_PANELS)
 *   person_counts n int64                                      (CSA_WANT_COUNTS)
 *   pair_counts   n * n int64, row-major; entries i < j and the
 *                 diagonal (= person_counts) are valid; the rest
 *                 is unspecified                               (CSA_WANT_PAIRS)
 *   unique_out    1 uint64 = number of distinct panels          (CSA_WANT_UNIQUE)
 *   attempts_out  n_panels uint32 attempts used per panel (>= 1), or NULL
 * max_attempts caps restarts per panel (0 = default 100000). */
int csa_legacy_sample(csa_instance *inst, int32_t k, uint64_t seed, uint64_t panel_begin,
                      uint64_t n_panels, uint32_t flags, uint32_t max_attempts,
                      uint64_t *panels_out, int64_t *person_counts, int64_t *pair_counts,
                      uint64_t *unique_out, uint32_t *attempts_out);

/* legacy_probabilities (analysis.py:162-191) over several devices of this process: the n_devices
 * argument of SURVEY.md §8(b)'s proposed csa_legacy_sample, for callers without torch.distributed.
 * Shard s (0 <= s < n_shards) draws the contiguous panel range
 *   [panel_begin + n_panels*s/n_shards, panel_begin + n_panels*(s+1)/n_shards)
 * on device devices[s] (NULL: device s; a device may repeat), on a replica of the instance that
 * the handle owns and keeps across calls (it mirrors csa_instance_set_state / _set_address).
 * Per-person and pair counts are summed on shard 0's device (peer copies + an add kernel); every
 * shard reduces its panels to its exact local distinct set and shard 0 counts the union exactly
 * (128-bit hash AND W-word bitmask).  Results are identical to csa_legacy_sample over the same
 * range for any n_shards and device list.  Arguments and outputs as csa_legacy_sample. */
int csa_legacy_sample_devices(csa_instance *inst, const int32_t *devices, int32_t n_shards, int32_t k,
                              uint64_t seed, uint64_t panel_begin, uint64_t n_panels, uint32_t flags,
                              uint32_t max_attempts, uint64_t *panels_out, int64_t *person_counts,
                              int64_t *pair_counts, uint64_t *unique_out, uint32_t *attempts_out);

/* legacy_find (analysis.py:141-159), batched: panels in pick order.
 * picks_out: n_panels * k int32 (a step that picked nobody -- only possible
 * with an inconsistent initial state -- is -1); attempts_out may be NULL. */
int csa_legacy_find(csa_instance *inst, int32_t k, uint64_t seed, uint64_t panel_begin,
                    uint64_t n_panels, uint32_t max_attempts, int32_t *picks_out,
                    uint32_t *attempts_out);

/* One call of find_random_sample_legacy (legacy.py:178-200) = one attempt
 * (seed, panel, attempt) from the instance's initial state.  Returns CSA_OK
 * (picks + final state written), CSA_E_SELECTION (SelectionError; state
 * outputs unspecified) or CSA_E_NO_CANDIDATE.  picks_out: k int32 in pick
 * order, *n_picks set; sel_out/rem_out: F; present_out: W (any may be NULL). */
int csa_legacy_attempt(csa_instance *inst, int32_t k, uint64_t seed, uint64_t panel,
                       uint32_t attempt, int32_t *picks_out, int32_t *n_picks, int32_t *sel_out,
                       int32_t *rem_out, uint64_t *present_out);

/* XMIN's LEGACY caller (_get_panel_not_in_portfolio_if_possible, xmin.py:464-474):
 * draw panels panel_begin, panel_begin+1, ... (at most n_panels; chunks of `chunk`
 * panels, doubling) and stop at the first one that is not in the portfolio (m packed
 * panels, host memory, m*W uint64; exact bitmask comparison behind a device hash
 * table).  *index_out = its offset from panel_begin (-1: all n_panels are members),
 * panel_out (W uint64) = that panel.  A draw error (KeyError / attempt limit) is
 * returned only if every panel before it is a member, as in the reference loop. */
int csa_first_panel_not_in(csa_instance *inst, int32_t k, uint64_t seed, uint64_t panel_begin,
                           uint64_t n_panels, uint32_t max_attempts, const uint64_t *portfolio,
                           uint64_t m, uint64_t chunk, int64_t *index_out, uint64_t *panel_out);

/* MT19937 mode (the reference's own stream), host only, no device
 * needed: `n_panels` consecutive legacy_find calls (analysis.py:141-159; single = 1: ONE
 * find_random_sample_legacy call, legacy.py:178-200, returning CSA_E_SELECTION on a dead end)
 * drawing from the stdlib random stream exactly as legacy.py:149 consumes it.  mt_state: 625
 * uint32 = CPython's random.getstate()[1] (624 words + position), advanced in place.  Instance
 * arrays as csa_instance_create; sel0 / rem0 (F) and present0 (W) give the start state (NULL =
 * 0 / pool counts / everyone), addr_next the same-address rings (or NULL, see
 * csa_instance_set_address).  Outputs (each may be NULL): picks_out n_panels*k (pick order, -1
 * padded), panels_out n_panels*W, attempts_out n_panels; with single, the final sel/rem (F) and
 * remaining pool (W); stats_out (3 uint64) the call's attempts, SelectionErrors and min-quota
 * rejections, as csa_instance_draw_stats counts them (a single attempt that raises counts one
 * SelectionError). */
int csa_legacy_draw_mt(int32_t n, int32_t C, int32_t F, const int32_t *person_feat, const int32_t *fmin,
                       const int32_t *fmax, const int32_t *sel0, const int32_t *rem0, const uint64_t *present0,
                       const int32_t *addr_next, int32_t k, uint32_t *mt_state, uint64_t n_panels,
                       uint32_t max_attempts, int32_t single, int32_t *picks_out, uint64_t *panels_out,
                       uint32_t *attempts_out, int32_t *sel_out, int32_t *rem_out, uint64_t *present_out,
                       uint64_t *stats_out);

/* ---- stream-ordered device API ---------------------------------------------
 * All buffers are device pointers on the instance's device; `stream` is a
 * hipStream_t (NULL = default stream).  Nothing synchronises; errors inside
 * kernels land in d_status (4 uint32: code, panel lo, panel hi, last attempt
 * result) which the caller zeroes before the first launch and decodes with
 * csa_status_decode after synchronising. */

/* Batch draw (analysis.py:141-159 per panel).  The instance's shape picks the kernel: a panel's
 * state (per-feature need / remaining keys and the remaining-pool bitset) lives in REGISTERS, split
 * over 1 lane (draw_solo_kernel, F <= 16), 2 lanes (draw_lane_kernel, F <= 32, n <= 2048) or 8
 * lanes (draw_wide_kernel, F <= 64, n <= 8192) of a wavefront, with the feature rows and person
 * masks in LDS; draw_kernel (16 or 64 lanes per panel) covers every other shape, pick orders and
 * same-address rings.  d_panels: n_panels*W (required); d_hashes: 2*n_panels 128-bit panel hashes
 * (or NULL); d_attempts: n_panels (or NULL); d_picks: n_panels*k (or NULL). */
/* Panels one full round of the batch draw's resident workgroups covers on the instance's device
 * (CUs x resident workgroups per CU x panels per workgroup, for this k): a csa_draw_async launch of
 * a multiple of it ends without a part-empty last round (callers that cut a batch into chunks use
 * it to size them).  *out = 0 on error. */
int csa_draw_round_panels(const csa_instance *inst, int32_t k, uint64_t *out);

int csa_draw_async(const csa_instance *inst, int32_t k, uint64_t seed, uint64_t panel_begin,
                   uint64_t n_panels, uint32_t max_attempts, uint64_t *d_panels,
                   uint64_t *d_hashes, uint32_t *d_attempts, int32_t *d_picks,
                   uint32_t *d_status, void *stream);
/* csa_draw_async that also writes the launch's panels as XT (d_xt: the csa_transpose_count_async
 * layout for n_panels, csa_xt_pad(n) persons per plane) when draw_lane_kernel runs with its fused pack
 * (*xt_written = 1): the caller then skips csa_transpose_count_async and takes the per-person counts
 * from the pair matrix's diagonal (csa_pairs_diag_async).  *xt_written = 0: d_xt untouched, the
 * panels / hashes as csa_draw_async.  flags: CSA_DRAW_RESET_STATUS / CSA_DRAW_RESET_STATS fold a
 * batch's resets into the same call (stream-ordered before the draw).  Replaces the separate transpose pass after one batch's draw
 * (analysis.py:179-190 count the same panels). */
#define CSA_DRAW_RESET_STATUS 0x1u /* csa_draw_xt_async flags: zero d_status (4 words) first, */
#define CSA_DRAW_RESET_STATS 0x2u  /* and this instance's draw statistics, on the stream */
int csa_draw_xt_async(const csa_instance *inst, int32_t k, uint64_t seed, uint64_t panel_begin,
                      uint64_t n_panels, uint32_t max_attempts, uint64_t *d_panels, uint64_t *d_hashes,
                      uint32_t *d_attempts, uint32_t *d_status, uint32_t *d_xt, int32_t *xt_written,
                      uint32_t flags, void *stream);

/* Re-draw panels [panel_begin, panel_begin + n_panels) exactly as csa_draw_async drew them (the same
 * kernel and Philox counters (seed, global panel index, attempt, step), so the same bitmasks), without
 * adding them to the instance's draw statistics.  A sharded run's found_panels (analysis.py:171,186;
 * pickled by run_legacy_or_retrieve, analysis.py:284-290) are re-made this way on whichever rank reads
 * them, instead of being gathered from the other ranks.  d_panels: n_panels*W; d_status as above. */
int csa_redraw_async(const csa_instance *inst, int32_t k, uint64_t seed, uint64_t panel_begin,
                     uint64_t n_panels, uint32_t max_attempts, uint64_t *d_panels, uint32_t *d_status,
                     void *stream);

/* The same draw split in two, for instances whose batch draw is the pick-list kernel
 * (draw_lane_kernel: F <= 32, n <= 2048; csa_draw_picks_supported returns 1 for them, else 0 and
 * csa_draw_picks_async returns CSA_E_UNSUPPORTED).  csa_draw_picks_async writes each panel's k
 * picks in pick order (legacy.py:194 people_selected order) into a row of
 * csa_picks_stride(k) = k rounded up to 8 uint16 (d_picks: n_panels * stride; entries past k
 * unspecified);
 * csa_picks_pack_async turns pick lists into packed panels (n_panels*W) and, if d_hashes is not
 * NULL, their 128-bit hashes.  csa_draw_async = the two back to back on one stream (with an
 * instance-owned pick buffer: concurrent csa_draw_async calls on one instance serialise). */
int32_t csa_picks_stride(int32_t k);
int csa_draw_picks_supported(const csa_instance *inst, int32_t k);
int csa_draw_picks_async(const csa_instance *inst, int32_t k, uint64_t seed, uint64_t panel_begin,
                         uint64_t n_panels, uint32_t max_attempts, uint16_t *d_picks, uint32_t *d_attempts,
                         uint32_t *d_status, void *stream);
int csa_picks_pack_async(const uint16_t *d_picks, uint64_t n_panels, int32_t k, int32_t n, uint64_t *d_panels,
                         uint64_t *d_hashes, void *stream);

/* 128-bit panel hashes (2*n_panels uint64) of packed panels (n_panels*W), the
 * key of the distinct-panel count (replaces hashing the sorted tuples of
 * analysis.py:171,186); identical to the hashes csa_draw_async writes. */
int csa_panel_hash_async(const uint64_t *d_panels, uint64_t n_panels, int32_t W, uint64_t *d_hashes,
                         void *stream);

/* Name of the draw kernel csa_draw_async launches for this instance and k
 * (e.g. "draw_lane_kernel<32, 28, 14>"), for matching profiler output. */
int csa_draw_kernel_name(const csa_instance *inst, int32_t k, char *buf, uint64_t len);

/* Bit-transpose + per-person count.  Panels (n_panels*W) -> d_xt, the
 * panel-indicator matrix transposed and packed in two 32-bit planes per
 * 64-panel block b (uint32 view): d_xt32[(2b + h) * n_pad + p] holds the bits
 * of agent p for panels 64b + 32h .. 64b + 32h + 31 (bit j = panel
 * 64b + 32h + j); n_pad = csa_xt_pad(n), blocks b < ceil(n_panels/64), i.e.
 * ceil(n_panels/64) * n_pad uint64 of storage.  The planes let the MFMA kernel
 * read every fragment bank-conflict-free.  d_counts (n int64) is ACCUMULATED
 * (+=); d_xt may be NULL (counts only). */
int32_t csa_xt_pad(int32_t n);
int csa_transpose_count_async(const uint64_t *d_panels, uint64_t n_panels, int32_t n,
                              uint64_t *d_xt, int64_t *d_counts, void *stream);

/* Pair counts X^T X on MFMA, upper-triangular 256x256 blocks (replaces
 * PairHistogram.add_portfolio_of_panels_to_histogram,
 * analysis.py:90-95, summed over all panels).  d_xt as produced above
 * (n_blocks = ceil(n_panels/64)); d_pairs (n*n int64, row-major) is
 * ACCUMULATED (+=) for i <= j (lower triangle unspecified).  Exact for any
 * n_blocks (each split stays inside its accumulator's exact integer range).
 * engine: CSA_PAIR_FP4 = v_mfma_scale_f32_32x32x64_f8f6f4 on e2m1 0/1-products
 * (f32 accumulation, exact below 2^24 per split); CSA_PAIR_I8 =
 * v_mfma_i32_32x32x32_i8 (int32 accumulation).  With d_scratch (at least
 * csa_pair_scratch_bytes bytes of device memory) the fp4 engine runs one
 * persistent workgroup per CU with the tiles grouped by XCD (whole tiles stored
 * directly, the leftover tiles as k-pieces summed by a reduce kernel; <= 2^24
 * panels per call, else as below); otherwise each split of the panel blocks
 * writes an int32 partial block that a reduce kernel sums, or, with d_scratch ==
 * NULL, adds into d_pairs with int64 atomics.  csa_pair_counts_async =
 * engine FP4, no scratch.  engine | CSA_PAIR_OVERWRITE stores instead of
 * accumulating: on return d_pairs holds exactly this batch's counts for i <= j
 * (the reduce kernel writes every element of the upper-triangular blocks; without
 * scratch the call zero-fills d_pairs first), so a caller that counts each batch
 * afresh needs no n*n zero-fill of its own.  engine | CSA_PAIR_SHARED is a
 * scheduling hint, never a change of result: the launch will share the CUs with
 * concurrent draw kernels (a pipelined caller).  The library currently takes the
 * same 512-register per-CU form either way (measured faster beside the draws than
 * the 256-register form, which CSA_P2_NB=2 still selects).  engine | CSA_PAIR_ALONE
 * is the opposite hint: nothing runs beside the launch (a serial caller's last
 * batch), so the kernel fastest alone is taken: the per-CU kernel from 2048 panel
 * blocks and 4 tiles per side (n > 768), the split kernel below (measured,
 * profiles/r06_pair_alone/). */
#define CSA_PAIR_FP4 0u
#define CSA_PAIR_I8 1u
#define CSA_PAIR_OVERWRITE 0x100u
#define CSA_PAIR_SHARED 0x200u
#define CSA_PAIR_ALONE 0x400u
uint64_t csa_pair_scratch_bytes(int32_t n, uint64_t n_blocks, uint32_t engine);
int csa_pair_counts_ex_async(const uint64_t *d_xt, uint64_t n_blocks, int32_t n, int64_t *d_pairs,
                             uint32_t engine, void *d_scratch, uint64_t scratch_bytes, void *stream);
int csa_pair_counts_async(const uint64_t *d_xt, uint64_t n_blocks, int32_t n, int64_t *d_pairs,
                          void *stream);

/* Distinct-panel count (found_panels, analysis.py:171,186): two panels are the same iff their
 * 128-bit hashes AND their W-word bitmasks are equal, so the count is exact.  d_panels (n_panels*W)
 * is required.  d_table: table_slots uint64 (power of two >= 2*n_panels) of scratch; *d_unique
 * (uint64) is ACCUMULATED.  With d_status (the 4-word status block) batches of >= 65536 panels take a
 * partitioned path (per-partition LDS tables, no per-panel global atomics); a partition table that
 * overflows sets CSA_E_UNSUPPORTED there.  With d_status == NULL the single global table runs. */
int csa_unique_async(const uint64_t *d_hashes, const uint64_t *d_panels, uint64_t n_panels, int32_t W,
                     uint64_t *d_table, uint64_t table_slots, uint64_t *d_unique, uint32_t *d_status,
                     void *stream);

/* Histogram of the pair counts d_pairs[i][j], i < j (n*n int64, row-major, as
 * produced by csa_pair_counts_*): d_hist[v] (n_bins uint64, zeroed by the call)
 * = number of pairs with count v; pairs with count >= n_bins are counted in
 * *d_overflow (zeroed by the call).  With n_bins = max person count + 1 nothing
 * overflows.  The sorted pair probabilities that
 * plot_pair_probability_distribution_per_algorithm (analysis.py:330-353) draws
 * are v / S repeated d_hist[v] times, v ascending. */
int csa_pair_histogram_async(const int64_t *d_pairs, int32_t n, uint64_t *d_hist, uint64_t n_bins,
                             uint64_t *d_overflow, void *stream);

/* Distinct panels over SEGMENTED input (the owner side of the multi-GPU exchange): n_segments
 * segments of `capacity` entries each (hashes 2*capacity, panels capacity*W uint64 per segment),
 * of which segment s holds d_seg_counts[s] (device uint64) valid leading entries.  Otherwise as
 * csa_unique_async: *d_unique += the exact distinct count; table_slots >= 2*n_segments*capacity. */
int csa_unique_segments_async(const uint64_t *d_hashes, const uint64_t *d_panels, uint32_t n_segments,
                              uint64_t capacity, const uint64_t *d_seg_counts, int32_t W, uint64_t *d_table,
                              uint64_t table_slots, uint64_t *d_unique, uint32_t *d_status, void *stream);

/* Multi-GPU distinct-panel exchange, send side (no host synchronisation; replaces the reference's
 * per-run `found_panels` set, analysis.py:171,186, across ranks).  The exact LOCAL distinct panels
 * of d_hashes / d_panels (n_panels, hash AND bitmask equality) are bucketed by owner rank
 * h1 % world into fixed-capacity segments: d_send_hashes uint64[world][capacity][2],
 * d_send_panels uint64[world][capacity][W], d_send_counts uint64[world] (entries per segment;
 * unused entries are left unwritten).  All three feed equal-split all_to_alls; the owner then calls
 * csa_unique_segments_async on what it received.  A segment that would exceed `capacity` raises
 * CSA_E_UNSUPPORTED in d_status (required).  d_scratch: csa_exchange_scratch_bytes(n_panels) bytes.
 * world <= 1024, n_panels < 2^31. */
uint64_t csa_exchange_scratch_bytes(uint64_t n_panels);
int csa_exchange_pack_async(const uint64_t *d_hashes, const uint64_t *d_panels, uint64_t n_panels, int32_t W,
                            uint32_t world, uint64_t capacity, void *d_scratch, uint64_t scratch_bytes,
                            uint64_t *d_send_hashes, uint64_t *d_send_panels, uint64_t *d_send_counts,
                            uint32_t *d_status, void *stream);

/* The 24-byte distinct-panel exchange.  A panel is a pure function of (seed, global panel index) in
 * the Philox stream, so instead of its bitmask each local distinct panel travels as a key
 * (h1, h2, panel_begin + local index).  Send side (as csa_exchange_pack_async otherwise):
 * d_send_keys uint64[world][capacity][3], scratch csa_exchange_scratch_bytes(n_panels).  Owner
 * side: *d_unique += the exact number of distinct panels among the valid keys of n_segments
 * segments of `capacity` keys (segment s holds d_seg_counts[s]): the distinct 128-bit hashes, plus
 * -- every key whose hash matched an earlier key being re-drawn on inst (draw over an index list,
 * Philox (k, seed, max_attempts) as the original draws) together with that key's panel -- the
 * mismatched ones (128-bit hash collisions) counted exactly by bitmask.  d_scratch:
 * csa_unique_keys_scratch_bytes(n_segments * capacity, W) bytes. */
int csa_exchange_keys_async(const uint64_t *d_hashes, const uint64_t *d_panels, uint64_t n_panels, int32_t W,
                            uint64_t panel_begin, uint32_t world, uint64_t capacity, void *d_scratch,
                            uint64_t scratch_bytes, uint64_t *d_send_keys, uint64_t *d_send_counts,
                            uint32_t *d_status, void *stream);
uint64_t csa_unique_keys_scratch_bytes(uint64_t n_keys, int32_t W);
int csa_unique_keys_async(const csa_instance *inst, int32_t k, uint64_t seed, uint32_t max_attempts,
                          const uint64_t *d_keys, uint32_t n_segments, uint64_t capacity,
                          const uint64_t *d_seg_counts, void *d_scratch, uint64_t scratch_bytes,
                          uint64_t *d_unique, uint32_t *d_status, void *stream);

/* Multi-GPU pair exchange: pack the upper triangle incl. the diagonal of the
 * n*n int64 pair counts row-major into n(n+1)/2 int32 (every count must be
 * < 2^31), and unpack it back (overwriting the upper triangle). */
int csa_pairs_pack_async(const int64_t *d_pairs, int32_t n, int32_t *d_packed, void *stream);
int csa_pairs_unpack_async(const int32_t *d_packed, int32_t n, int64_t *d_pairs, void *stream);

/* PairHistogram materialisation (replaces the host-side division and triangle walk of
 * analysis.py:86-98): the strict upper triangle (i < j, row-major -- the reference's key order,
 * analysis.py:70) of the n*n int64 pair counts, packed into n(n-1)/2 entries of d_out: float64
 * count / divisor (IEEE, correctly rounded: Python's int / int) for divisor > 0, int64 counts for
 * divisor == 0.  Stream-ordered. */
int csa_pairs_upper_async(const int64_t *d_pairs, int32_t n, double divisor, void *d_out, void *stream);

/* Per-person counts (agent_appearance_counter, analysis.py:179, 187) = the diagonal of the n*n int64
 * pair counts (every panel contributes x_i * x_i = x_i): d_counts[i] = d_pairs[i*n + i] (stored). */
int csa_pairs_diag_async(const int64_t *d_pairs, int32_t n, int64_t *d_counts, void *stream);

/* Decode a device status block (host copy of the 4 words) into a CSA_* code
 * and set csa_last_error() accordingly. */
int csa_status_decode(const uint32_t *h_status);

#ifdef __cplusplus
}
#endif
#endif /* CSA_LEGACY_H */
