/* bwagpu_debug.h — tuning, test and profiling entry points of libbwagpu.so.
 *
 * Not part of the drop-in stage's interface (include/bwagpu.h): bwa-flow's
 * ChainsToRegionsGPU never calls them.  The tests use them to force kernel
 * forms and inject failures, and bench.py uses them to time the dominant
 * extension kernel (HIP events) and read the speculative path's counters.
 * The reference has no counterpart: it logs per-phase stage wall times
 * (src/fpga/FPGAPipeline.cpp:557-578, src/util.h:34-40).  Every entry here
 * leaves results unchanged.
 */
#ifndef BWAGPU_DEBUG_H
#define BWAGPU_DEBUG_H
#include "bwagpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Tuning / tests: bwagpu_collect_intv runs each read on one lane until it has
   made `budget` bwt_extend calls (default 1024, about the 90th percentile of a
   150 bp read on a chr21-sized index), then hands it to a second kernel that
   runs it on a whole wave (backward search lane-parallel).  0 sends every
   read to the wave kernel.  Results do not depend on it. */
int bwagpu_debug_seed_budget(bwagpu_ctx_t *ctx, int32_t budget);

/* Tests: the device occurrence layout keeps 32-bit counts relative to
   superblocks of 2^shift positions (default 32: only indexes past 2^32
   positions, e.g. GRCh38's 6.2 G, have more than one).  A smaller shift
   (7..32) for the NEXT bwagpu_set_bwt makes a small index cross superblock
   boundaries, so that the superblock table and the relative counts are
   exercised on the golden fixtures.  Results do not depend on it. */
int bwagpu_debug_sup_shift(bwagpu_ctx_t *ctx, int32_t shift);

/* diagnostics: while dev_ptr != NULL every chain2aln launch on this device
   writes 8 x uint32 per read index r at dev_ptr[8r..8r+7]: start and end
   s_memrealtime (100 MHz, lo/hi), DP rows, DP cells, HW_ID, XCC_ID (the
   per-read kernels); the speculative path writes its selection passes
   (emulate, final, redo) at dev_ptr[8 (pass n_reads + r) ..]: start / end,
   seeds, regions, XCC_ID, shape — so the buffer needs 24 x n_reads words.
   Not part of the reference interface (the reference logs stage wall times
   with getUs(), src/util.h:34-40). */
int bwagpu_debug_set_trace(bwagpu_ctx_t *ctx, void *dev_ptr);
/* tests of the caller's recovery path: after `after_n_waits` more successful
   bwagpu_chain2aln_wait calls, the next one returns `code` (e.g.
   BWAGPU_E_HANG, as a watchdog expiry does) with its batch left in flight */
int bwagpu_debug_fail_wait(bwagpu_ctx_t *ctx, int after_n_waits, int code);

/* kernel timing (bench.py's roofline): after bwagpu_prof_start(ctx, n) the
   next n launches of the dominant extension kernel (the first length bin's
   extension kernel, one per extension round of a chain2aln batch) are
   bracketed by HIP events on the stream they run on; bwagpu_prof_read waits
   for them and returns the summed kernel time and the number of launches
   timed; bwagpu_prof_intervals returns each launch's [start, end] in ms from
   the first event, so that launches of different streams that overlap can be
   counted once (their union).  bwagpu_prof_start(ctx, 0)
   turns timing off.  Diagnostics; the reference prints per-phase stage times
   instead (src/fpga/FPGAPipeline.cpp:557-578). */
int bwagpu_prof_start(bwagpu_ctx_t *ctx, int max_launches);
/* diagnostics: the speculative path's counters of the last device-entry batch
   on `stream` (waits for it): out[0..2] extension tasks of rounds A/B/C,
   out[3] DP cells of every computed task (used or not), out[4] extensions the
   redo pass computed inline, out[5] reads with > 64 seeds, out[6] reads left
   to the redo pass, out[7] seeds of heavy reads with pair matrices */
int bwagpu_debug_spec_counters(bwagpu_ctx_t *ctx, void *stream, int64_t *out);
/* diagnostics of a library built with -DBWAGPU_OCC_DIAG (else
   BWAGPU_E_UNSUPPORTED): the packed extension kernels' occupancy over the last
   device-entry batch on `stream`, out[0..7] = generations (extend_quad calls
   of a wave), rows run, call-slot rows, live call rows, call-slot cells, live
   call-slot cells, cells inside the live calls' queries, computed cells;
   out[8..11] = the waves' shader-clock cycles in task starts + claims, call
   setup, the DP (extend_quad) and the result advance, out[12..13] = of the
   first, the claims' and the task records' own (out: 14 entries) */
int bwagpu_debug_occupancy(bwagpu_ctx_t *ctx, void *stream, int64_t *out);
/* diagnostics: the per-seed extension records (48 B each: rb, re, qb, qe,
   score, truesc, w, cells, rows, calls + 1; calls == 0: not computed) of the
   last device-entry batch on `stream`, n = its seed count */
int bwagpu_debug_spec_ext(bwagpu_ctx_t *ctx, void *stream, void *host_out, int32_t n);
int bwagpu_prof_read(bwagpu_ctx_t *ctx, double *total_ms, int32_t *launches);
/* tests / A-B: the extension kernel of the first two read-length bins — 0
   (default) packed 16-bit DP where every score of the bin fits (else two per
   wave): eight seeds per wave in the first bin, four in the second; 1 two
   seeds per wave (32-bit DP); 2 four seeds per wave in both bins.  Results do
   not depend on it.  bwagpu_ctx_ext_form sets one context's form;
   bwagpu_debug_ext_form sets the form contexts created afterwards start with.
   Both return the previous form; form < 0 only queries. */
int bwagpu_debug_ext_form(int form);
int bwagpu_ctx_ext_form(bwagpu_ctx_t *ctx, int form);
/* the packed extension kernels' row bound (default on): a ksw_extend2 call
   ends once no later target row can change its score, qle, tle, gtle, gscore
   or max_off (every later cell is bounded by a stored value plus max(mat) per
   query column still ahead of it).  Results are identical either way; with
   it off the cell and row counters (bwagpu_last_stats) count every row
   ksw_extend2 (ksw.c:380-479) evaluates.  Returns the previous setting;
   on < 0 only queries. */
int bwagpu_ctx_row_bound(bwagpu_ctx_t *ctx, int on);
/* the first length bin's extension kernel this context launches for reads of
   up to lq_max bases: 8 = eight seeds per wave (spec_ext4_kernel<16,10,true>),
   4 = four per wave with the 8-bit row-max key (<32,5,true>), 5 = four per
   wave (<32,8,false>), 2 = two per wave (spec_ext2_kernel<5>); 18 / 14 / 15 =
   the same shapes as the phased pair spec_side4_kernel<G,PMAX,K8,{false,true}>
   (every left call, then every right call; BWAGPU_EXT_PHASED bit 0); 28 = the
   eight-per-wave pair with a producer wave, spec_sidep_kernel<16,10,true,*>
   (BWAGPU_EXT_PRODUCER) */
int bwagpu_debug_ext_kernel(bwagpu_ctx_t *ctx, int32_t lq_max);
/* 1 if work on the two streams (hipStream_t, on the current device) runs
   concurrently, 0 if they share a hardware queue (HIP maps the process's
   streams onto GPU_MAX_HW_QUEUES queues; streams on one queue run in
   submission order), < 0 on error.  Measured: a ~150 us spin on a, then an
   empty kernel on b.  Callers that drive several batches at once should give
   them concurrent streams (bench.py's caller_streams). */
int bwagpu_streams_concurrent(void *a, void *b);
int bwagpu_prof_intervals(bwagpu_ctx_t *ctx, double *start_ms, double *end_ms, int32_t max, int32_t *n);

#ifdef __cplusplus
}
#endif
#endif /* BWAGPU_DEBUG_H */
