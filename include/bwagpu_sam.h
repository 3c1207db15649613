/*
 * bwagpu_sam.h — C ABI of the SAM-stage call cache (lib/libgpusam.so).
 *
 * bwa-flow's SAM stage (RegionsToSam, src/Pipeline.cpp:546-648) runs bwa's
 * mem_sam_pe per pair (Pipeline.cpp:584-600).  Inside it, two kinds of calls
 * carry the Smith-Waterman work:
 *
 *   ksw_align2   mate rescue, from mem_matesw (bwa/bwamem_pair.c:154), replaced
 *                by bwagpu_align2_batch;
 *   mem_reg2aln  CIGAR + MD + NM of each printed region (bwa/bwamem.c:1104-1174,
 *                called from bwamem_pair.c:343/351/382, bwamem.c:1037 and
 *                bwamem_extra.c:119; bwa-flow's copies at src/bwa_wrapper.cpp:
 *                611/728/736/774), replaced by bwagpu_reg2aln_batch.
 *
 * Which calls a pair makes depends on earlier results (a rescued hit can make
 * a later rescue redundant, bwamem_pair.c:123-128; the printed regions depend
 * on the rescues), so the calls cannot be listed up front.  The cache turns
 * the record's mem_sam_pe loop into collect -> batch -> replay passes:
 *
 *   1. run the loop on a copy of the record's regions with the two functions
 *      interposed (bwa-flow_amd/host/sam_hooks.c): every call looks itself up
 *      in the cache; a miss queues the call and answers with a placeholder
 *      (no rescue hit / a region without CIGAR), so the pass runs to the end;
 *   2. bwagpu_samcache_flush: the queued calls go to the device in one
 *      bwagpu_align2_batch and one bwagpu_reg2aln_batch;
 *   3. repeat until a pass has no miss: that pass's SAM text is the output,
 *      byte-identical to the CPU stage's.  Typically three passes: rescues
 *      missed, then CIGARs of the final regions missed, then none.
 *
 * Calls are keyed by their full content (bases, window, band, flags), so
 * passes may run on any number of threads in any order.  All functions are
 * thread-safe except _flush, _clear and _destroy, which need the stage's
 * worker threads joined.
 */
#ifndef BWAGPU_SAM_H
#define BWAGPU_SAM_H

#include "bwagpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct bwagpu_samcache bwagpu_samcache_t;

/* a cache whose flushes run on ctx (its opt is the stage's mem_opt_t: mat,
   gap penalties, a, w).  max_ops / max_md: the per-call CIGAR-op and MD-byte
   capacity of the first reg2aln launch; calls that overflow it are re-run with
   room for any alignment of their read. */
int bwagpu_samcache_create(bwagpu_ctx_t *ctx, int32_t max_ops, int32_t max_md, bwagpu_samcache_t **out);
int bwagpu_samcache_destroy(bwagpu_samcache_t *c);
/* forget every entry (between records) */
int bwagpu_samcache_clear(bwagpu_samcache_t *c);

/* ksw_align2(qlen, query, tlen, target, 5, mat, o_del, e_del, o_ins, e_ins,
   xtra, 0) with query/target in 0..4.  Returns 0 on a hit (*out = that call's
   kswr_t) or 1 on a miss (the call is queued; *out = {0, -1, -1, -1, -1, -1,
   -1}, which mem_matesw treats as "no hit", bwamem_pair.c:155), or a negative
   BWAGPU_E_* code on a bad argument. */
int bwagpu_samcache_align2(bwagpu_samcache_t *c, int32_t qlen, const uint8_t *query, int32_t tlen,
                           const uint8_t *target, int32_t xtra, bwagpu_kswr_t *out);

/* mem_reg2aln's CIGAR part for a mapped region (rb >= 0, re >= 0) of a read
   of l_seq nt4 bases.  On a hit returns 0, *out = the job's bwagpu_aln_t and
   *cigar = a malloc'd block of out->n_cigar ops followed by the NUL-terminated
   MD string (mem_aln_t.cigar's layout, bwamem.c:1137-1166; the caller frees
   it).  On a miss returns 1, queues the job, sets out->status = -1 and *cigar
   to a malloc'd empty block (no ops, MD "").  Negative BWAGPU_E_* on error. */
int bwagpu_samcache_reg2aln(bwagpu_samcache_t *c, int32_t l_seq, const uint8_t *read, int64_t rb, int64_t re,
                            int32_t qb, int32_t qe, int32_t truesc, int32_t w, bwagpu_aln_t *out,
                            uint32_t **cigar);

/* runs every queued call on the device.  Returns the number of calls computed
   (0 = nothing was queued: the last pass had no miss) or a negative BWAGPU_E_*
   code (bwagpu_last_error(ctx) says why). */
int64_t bwagpu_samcache_flush(bwagpu_samcache_t *c);

/* [0] align2 hits [1] align2 misses [2] reg2aln hits [3] reg2aln misses
   [4] align2 calls computed [5] reg2aln calls computed [6] flushes
   [7] flush wall time, microseconds */
int bwagpu_samcache_stats(const bwagpu_samcache_t *c, int64_t out[8]);

#ifdef __cplusplus
}
#endif
#endif
