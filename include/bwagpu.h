/*
 * bwagpu.h — C ABI of the MI355X seed-extension engine.
 *
 * This is the drop-in boundary that takes the place of bwa-flow's FPGA
 * Smith-Waterman back end (the files under src/fpga/).  Everything crossing it is plain C:
 * POD structs, pointers and sizes, integer return codes, no exceptions.
 *
 * What each entry point replaces in the reference (file:line into
 * falcon-computing/bwa-flow):
 *
 *   bwagpu_create / bwagpu_create_resident
 *       BWAOCLEnv::BWAOCLEnv + initPAC (src/fpga/BWAOCLEnv.h:41-114): bring up
 *       one device, make the 2-bit reference resident on it.  The reference
 *       uploads a forward+revcomp pac with a blocking clEnqueueWriteBuffer per
 *       device (BWAOCLEnv.h:92, 293-312); here only bwa's forward pac
 *       (bwa.c:281-282 layout, bntseq.c:225 bit order) is resident and the
 *       reverse strand is computed in-kernel.  _resident takes a pac that is
 *       already in HBM (e.g. broadcast over xGMI with RCCL by the host).
 *   bwagpu_chain2aln_submit
 *       SWTask::start -> XCLAgent::writeInput + clEnqueueTask(sw_top)
 *       (src/fpga/SWTask.cpp:106-152, xlnx/XCLAgent.cpp:51,89-106): stage one
 *       packed read batch into a slot's buffers and launch asynchronously.
 *   bwagpu_chain2aln_wait
 *   bwagpu_chain2aln_stage / _results (zero-copy host path)
 *       SWTask::finish -> XCLAgent::readOutput + processOutput
 *       (SWTask.cpp:154-180, XCLAgent.cpp:64, FPGAPipeline.cpp:29-130): wait
 *       with a watchdog and return finished mem_alnreg_t records.
 *   bwagpu_chain2aln
 *       submit + wait; the per-batch body of ChainsToRegionsFPGA::compute
 *       (FPGAPipeline.cpp:367-579) with the semantics of the CPU stage
 *       ChainsToRegions::compute (src/Pipeline.cpp:503-544) ->
 *       mem_chain2aln (bwa/bwamem.c:641-795) for every chain of every read.
 *   bwagpu_chain2aln_device
 *       the same launch with every input/output already in device memory
 *       (benchmarks, multi-stream hosts).
 *   bwagpu_extend_batch
 *       a batch of independent ksw_extend2 calls (bwa/ksw.c:380-479); the
 *       task-level granularity of the FPGA kernel's seed_proc
 *       (src/fpga/kernel/smithwaterman.cpp:318-445) but with ksw_extend2's
 *       exact semantics (z-drop, band trimming, runtime scoring).
 *   bwagpu_align2_batch
 *       a batch of independent ksw_align2 calls (bwa/ksw.c:337-357: ksw_u8 /
 *       ksw_i16 local SW, 2nd-best score, start by the reverse pass) as made
 *       by mate rescue, mem_matesw (bwa/bwamem_pair.c:150-151), for every
 *       read pair of a batch (mem_sam_pe, bwamem_pair.c:290-300).  Results
 *       equal ksw_align2's kswr_t field for field, including the quirks of
 *       its striped first pass (see oracle/ksw_align.c).
 *   bwagpu_sw_stream
 *       the FPGA kernel's own job, sw_top over one packed task stream
 *       (clEnqueueTask, xlnx/XCLAgent.cpp:89-106): the input stream of
 *       packReadData (src/fpga/FPGAPipeline.cpp:252-336) in, the 5-int
 *       per-seed result records processOutput reads (FPGAPipeline.cpp:90-105)
 *       out, every seed extended as mem_chain2aln extends one seed
 *       (bwa/bwamem.c:717-792) in its chain's window rmax.
 *   bwagpu_set_bwt / bwagpu_collect_intv / bwagpu_bwt_sa
 *       seeding's interval search and SA lookups for a batch (bwa_idx_load's
 *       bwt_t, mem_collect_intv bwamem.c:120-167, bwt_sa bwt.c:86-96).
 *   bwagpu_seqs2chains
 *       SeqsToChains' per-read body (src/bwa_wrapper.cpp:118-131: mem_chain,
 *       mem_chain_flt, mem_flt_chained_seeds) for a whole batch.
 *   bwagpu_seqs2regions
 *       SeqsToChains + ChainsToRegions (src/Pipeline.cpp:110-121, 503-544) as
 *       one device call: reads in, mem_alnreg_v out.
 *   bwagpu_last_error
 *       the what() of fpgaHangError / fpgaResultsError / std::runtime_error
 *       (src/util.h:16-32, OpenCLEnv.h:21-31).
 *   bwagpu_destroy
 *       BWAOCLEnv::~BWAOCLEnv (main.cpp:376-387).
 *
 * Results are bit-identical to the reference CPU path: every field that
 * mem_chain2aln writes (rb,re,qb,qe,rid,score,truesc,w,seedcov,seedlen0,
 * frac_rep), all other fields zero, regions in the same order.
 */
#ifndef BWAGPU_H
#define BWAGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BWAGPU_ABI_VERSION 1

/* return codes */
enum {
  BWAGPU_OK = 0,
  BWAGPU_E_INVAL = 1,       /* bad argument / malformed batch                       */
  BWAGPU_E_NOMEM = 2,       /* host or device allocation failed (FPGAPipeline.cpp:383-391) */
  BWAGPU_E_DEVICE = 3,      /* HIP runtime error (OpenCLEnv.h:21-31 analogue)       */
  BWAGPU_E_HANG = 4,        /* watchdog expired (fpgaHangError, SWTask.cpp:116-122)  */
  BWAGPU_E_RESULTS = 5,     /* device flagged an inconsistent input/result
                               (fpgaResultsError, FPGAPipeline.cpp:72; also the
                               reference's assert(c->rid == rid), bwamem.c:669)     */
  BWAGPU_E_UNSUPPORTED = 6, /* read longer than BWAGPU_MAX_READ_LEN                  */
  BWAGPU_E_NODEVICE = 7     /* no HIP device / not built for this device             */
};

/* longest read (bp) the device kernels accept; longer reads -> E_UNSUPPORTED */
#define BWAGPU_MAX_READ_LEN 1023
/* number of independent in-flight slots per context (ping-pong, FPGAPipeline.cpp:373-386) */
#define BWAGPU_NUM_SLOTS 4

/* The fields of mem_opt_t (bwa/bwamem.h:26-58) that mem_chain2aln/ksw_extend2 read. */
typedef struct {
  int32_t a, b;          /* match score, mismatch penalty (used by cal_max_gap)   */
  int32_t o_del, e_del;  /* deletion open/extend                                  */
  int32_t o_ins, e_ins;  /* insertion open/extend                                 */
  int32_t pen_clip5, pen_clip3;
  int32_t w;             /* band width                                            */
  int32_t zdrop;         /* z-dropoff                                             */
  int8_t mat[25];        /* 5x5 scoring matrix (bwa_fill_scmat, bwa/bwa.c:109-118) */
  int8_t pad_[3];
} bwagpu_opt_t;

/* == mem_seed_t (src/bwa_wrapper.h:62-66, bwa/bwamem.c:174-178), 24 bytes */
typedef struct {
  int64_t rbeg;
  int32_t qbeg, len;
  int32_t score;
  int32_t pad_;
} bwagpu_seed_t;

/* == mem_alnreg_t (bwa/bwamem.h:60-79), 88 bytes, same offsets */
typedef struct {
  int64_t rb, re;
  int32_t qb, qe;
  int32_t rid;
  int32_t score, truesc, sub, alt_sc, csub, sub_n;
  int32_t w, seedcov, secondary, secondary_all, seedlen0;
  uint32_t n_comp_is_alt; /* n_comp:30, is_alt:2 — always 0 from mem_chain2aln */
  float frac_rep;
  uint64_t hash;
} bwagpu_alnreg_t;

/* The parts of bntseq_t (bwa/bntseq.h:55-66) the path reads. */
typedef struct {
  int64_t l_pac;
  int32_t n_seqs;
  int32_t pad_;
  const int64_t *ann_offset; /* [n_seqs] bntann1_t.offset */
  const int32_t *ann_len;    /* [n_seqs] bntann1_t.len    */
} bwagpu_bns_t;

/*
 * One read batch (one ChainsRecord, src/Pipeline.h:46-57) in flattened form.
 * Read r has l_seq = seq_off[r+1]-seq_off[r] nt4 bases (0..4, already
 * converted in place as bwa_wrapper.cpp:124-125 does), chains
 * read_chain_off[r] .. read_chain_off[r+1]-1; chain c has seeds
 * chain_seed_off[c] .. chain_seed_off[c+1]-1 in mem_chain_t order, its
 * mem_chain_t.rid and .frac_rep.
 * Output: the regions of read r are written to
 *   out_regs[chain_seed_off[read_chain_off[r]] + k], k < out_n[r]
 * (a read never yields more regions than it has seeds), in the order
 * mem_chain2aln appends them to the read's mem_alnreg_v.
 */
typedef struct {
  int32_t n_reads, n_chains, n_seeds, pad_;
  int64_t seq_bytes;
  const int64_t *seq_off;        /* [n_reads+1]  */
  const uint8_t *seq;            /* [seq_bytes]  */
  const int32_t *read_chain_off; /* [n_reads+1]  */
  const int32_t *chain_seed_off; /* [n_chains+1] */
  const int32_t *chain_rid;      /* [n_chains]   */
  const float *chain_frac_rep;   /* [n_chains]   */
  const bwagpu_seed_t *seeds;    /* [n_seeds]    */
} bwagpu_batch_t;

/* One ksw_extend2 call: query = qpool[qoff..qoff+qlen), target = tpool[toff..toff+tlen). */
typedef struct {
  int64_t qoff, toff;
  int32_t qlen, tlen;
  int32_t w, end_bonus, zdrop, h0;
} bwagpu_ext_task_t;

/* ksw_extend2 outputs: return value and *qle,*tle,*gtle,*gscore,*max_off */
typedef struct {
  int32_t score, qle, tle, gtle, gscore, max_off;
} bwagpu_ext_result_t;

/* ksw_align2 xtra flags (bwa/ksw.h:6-9); the low 16 bits carry minsc/endsc */
#define BWAGPU_KSW_XBYTE 0x10000
#define BWAGPU_KSW_XSTOP 0x20000
#define BWAGPU_KSW_XSUBO 0x40000
#define BWAGPU_KSW_XSTART 0x80000

/* One ksw_align2(qlen, query, tlen, target, 5, opt->mat, opt->o_del, opt->e_del,
   opt->o_ins, opt->e_ins, xtra, 0) call: query = qpool[qoff..qoff+qlen),
   target = tpool[toff..toff+tlen).  qlen <= BWAGPU_MAX_READ_LEN. */
typedef struct {
  int64_t qoff, toff;
  int32_t qlen, tlen;
  int32_t xtra, pad_;
} bwagpu_align2_task_t;

/* == kswr_t (bwa/ksw.h:17-21); unset fields are -1 */
typedef struct {
  int32_t score, te, qe, score2, te2, tb, qb;
} bwagpu_kswr_t;

/* One mem_reg2aln CIGAR job (bwa/bwamem.c:1104-1174, as called per output
   region from src/bwa_wrapper.cpp:611/728/736/774): the region's
   rb/re/qb/qe/truesc/w (mem_alnreg_t) and its read, l_seq nt4 bases at
   qpool[qoff..qoff+l_seq).  rb < 0 or re < 0 asks for the unmapped record. */
typedef struct {
  int64_t rb, re;
  int64_t qoff;
  int32_t l_seq, qb, qe;
  int32_t truesc, w;
  int32_t pad_;
} bwagpu_reg2aln_task_t;

#define BWAGPU_ALN_OK 0
#define BWAGPU_ALN_NO_CIGAR 1 /* bwa_gen_cigar2 returned no CIGAR (bwa.c:133/135): the
                                 reference's mem_reg2aln would dereference NULL here */
#define BWAGPU_ALN_OVERFLOW 2 /* more than max_ops CIGAR ops or max_md MD bytes */
#define BWAGPU_ALN_UNMAPPED 3 /* rb < 0 || re < 0: rid = -1, pos = -1 (bwamem.c:1112-1115) */

/* The alignment fields mem_reg2aln fills in mem_aln_t (bwa/bwamem.h:81-92)
   besides mapq/flag/sub/alt_sc (which need the other regions): CIGAR with
   soft clips (ops at cigar[k * max_ops], BAM encoding len << 4 | op), the MD
   string after it in the reference layout (here at md[k * max_md],
   NUL-terminated, md_len = strlen), NM, strand, contig and 0-based position.
   score / w: the global score and band of the last bwa_gen_cigar2 call. */
typedef struct {
  int64_t pos;
  int32_t rid, is_rev;
  int32_t n_cigar, NM;
  int32_t md_len, score;
  int32_t w, status;
} bwagpu_aln_t;

/* ---- seeding: mem_collect_intv on the device ---- */

/* The FM-index of the reference as bwa holds it (bwt_t, bwa/bwt.h:46-57):
   primary, the cumulative counts L2[5], seq_len, and the bwt_size uint32
   words of the interleaved occurrence array (per 128 BWT positions: 4 uint64
   counts, then 8 words of 2-bit bases, first base in the highest bits). */
typedef struct {
  uint64_t primary;
  uint64_t L2[5];
  uint64_t seq_len;
  uint64_t bwt_size;
  const uint32_t *bwt;
  /* the sampled suffix array (bwt.h:55-57): sa[i] = SA[i * sa_intv], n_sa
     entries; sa may be NULL when bwagpu_bwt_sa is not used */
  int32_t sa_intv;
  int32_t pad_;
  uint64_t n_sa;
  const uint64_t *sa;
} bwagpu_bwt_t;

/* == bwtintv_t (bwa/bwt.h:60-62): x[0] / x[1] the SA intervals of the match
   and of its reverse complement, x[2] their size, info = start << 32 | end */
typedef struct {
  uint64_t x[3];
  uint64_t info;
} bwagpu_intv_t;

/* mem_opt_t's seeding fields (bwa/bwamem.h:34-46, defaults bwamem.c:62-72) */
typedef struct {
  int32_t min_seed_len; /* -k, 19 */
  int32_t split_width;  /* 10 */
  int32_t max_mem_intv; /* 20: the LAST-like third pass runs when > 0 */
  float split_factor;   /* -r, 1.5 */
} bwagpu_seedopt_t;

#define BWAGPU_MAX_SEED_READ 4096 /* longest read bwagpu_collect_intv takes */

/* mem_opt_t's chaining fields (bwa/bwamem.h:38-52, defaults bwamem.c:62-72);
   the band (w) and scoring (a, mat, gaps) come from the context's
   bwagpu_opt_t, min_seed_len from bwagpu_seedopt_t */
typedef struct {
  int32_t max_occ;          /* -c, 500: SA positions taken per interval  */
  int32_t max_chain_gap;    /* 10000                                     */
  int32_t min_chain_weight; /* 0                                         */
  int32_t max_chain_extend; /* 1<<30                                     */
  float mask_level;         /* 0.50                                      */
  float drop_ratio;         /* -D, 0.50                                  */
} bwagpu_chainopt_t;

/* one chain: mem_chain_t (bwa/bwamem.c:180-186) without its seed vector —
   the seeds follow in the batch layout (chain_seed_off / seeds) */
typedef struct {
  int64_t pos;      /* the first seed's rbeg: the kbtree key            */
  int32_t rid;      /* contig                                           */
  int32_t n;        /* seeds                                            */
  int32_t w;        /* mem_chain_weight (29-bit field)                  */
  int32_t kept;     /* mem_chain_flt: 1, 2 or 3 (0 chains are dropped)  */
  int32_t first;    /* mem_chain_flt's shadowed-chain index, -1 if none */
  int32_t is_alt;
  float frac_rep;
  int32_t pad_;
} bwagpu_chain_t;

/* per-launch statistics of the last finished launch on a slot */
typedef struct {
  double kernel_ms;      /* HIP-event time of the extension kernel(s)            */
  double total_ms;       /* H2D + kernel + D2H wall (submit..wait)               */
  int64_t cells;         /* evaluated DP cells: sum over executed rows of
                            (end-beg) as ksw.c:424 counts them.  Equal to the
                            reference's count only with the row bound off
                            (bwagpu_ctx_row_bound(ctx, 0), bwagpu_debug.h); with it on (the
                            default) the rows it skips are not counted, so
                            cells and rows fall below the reference's          */
  int64_t rows;          /* executed DP rows (the same caveat)                   */
  int64_t ext_calls;     /* ksw_extend2-equivalent calls                         */
  int64_t h2d_bytes, d2h_bytes;
} bwagpu_stats_t;

typedef struct bwagpu_ctx bwagpu_ctx_t;

int bwagpu_abi_version(void);
int bwagpu_device_count(int *n);

int bwagpu_create(int device, const bwagpu_opt_t *opt, const bwagpu_bns_t *bns,
                  const uint8_t *pac_host, bwagpu_ctx_t **ctx);
int bwagpu_create_resident(int device, const bwagpu_opt_t *opt, const bwagpu_bns_t *bns,
                           const void *pac_device, bwagpu_ctx_t **ctx);
int bwagpu_destroy(bwagpu_ctx_t *ctx);
const char *bwagpu_last_error(const bwagpu_ctx_t *ctx);

/* watchdog for _wait in milliseconds (default 10000, SWTask.cpp:116-122); 0 = none */
int bwagpu_set_watchdog_ms(bwagpu_ctx_t *ctx, int ms);

/* _wait returns BWAGPU_E_RESULTS when a chain's first seed lies outside its
   contig (where bwa asserts, bwamem.c:669); the outputs are still written:
   that chain is skipped, every other chain's regions are valid. */
int bwagpu_chain2aln_submit(bwagpu_ctx_t *ctx, int slot, const bwagpu_batch_t *batch);
int bwagpu_chain2aln_wait(bwagpu_ctx_t *ctx, int slot, bwagpu_alnreg_t *out_regs, int32_t *out_n);
int bwagpu_chain2aln(bwagpu_ctx_t *ctx, const bwagpu_batch_t *batch, bwagpu_alnreg_t *out_regs,
                     int32_t *out_n);

/* Zero-copy host path (packReadData writing straight into the device's DMA
   buffer instead of a staging copy, FPGAPipeline.cpp:252-336 / SWTask.cpp:
   writeInput).  _stage sizes the slot's pinned input buffer for a batch of
   these counts and fills *view with pointers into it (and the counts); the
   caller writes the batch there and passes *view to _submit, which then skips
   its copy.  The view stays valid until the slot's next _stage.  After a
   successful _wait(ctx, slot, NULL, NULL), _results points *regs / *n at the
   slot's pinned output (same layout as _wait's out_regs / out_n), valid until
   the slot's next _submit. */
int bwagpu_chain2aln_stage(bwagpu_ctx_t *ctx, int slot, int32_t n_reads, int32_t n_chains, int32_t n_seeds,
                           int64_t seq_bytes, bwagpu_batch_t *view);
int bwagpu_chain2aln_results(bwagpu_ctx_t *ctx, int slot, const bwagpu_alnreg_t **regs, const int32_t **n);
/* The same results as the device returns them: read r's n[r] regions at
   regs[off[r] .. off[r] + n[r]) (off[r] = n[0] + ... + n[r-1], off has n_reads
   + 1 entries), i.e. processOutput's order without the slot gaps
   (FPGAPipeline.cpp:29-130).  Only these bytes cross PCIe; _results and
   _wait's out_regs rebuild the slot layout from them on the host.  Valid until
   the slot's next _submit. */
int bwagpu_chain2aln_results_dense(bwagpu_ctx_t *ctx, int slot, const bwagpu_alnreg_t **regs, const int32_t **n,
                                   const int32_t **off);
/* all pointers in dev_batch / dev_out / dev_n are device pointers; stream is a
   hipStream_t (NULL = the context's slot-0 stream); asynchronous; dev_stats
   (device, 4 x int64: cells, rows, ext_calls, error flag) may be NULL.
   Up to BWAGPU_NUM_SLOTS distinct streams may be used on one context (each
   keeps its own scratch), so consecutive batches can overlap.  Two calls on
   the SAME stream are ordered by it; the device entry's scratch is separate
   from the submit/wait slots', so both entry points may be used concurrently
   on one context.  Options whose LDS need exceeds a launch are refused with
   BWAGPU_E_UNSUPPORTED before anything is enqueued. */
int bwagpu_chain2aln_device(bwagpu_ctx_t *ctx, const bwagpu_batch_t *dev_batch,
                            bwagpu_alnreg_t *dev_out, int32_t *dev_n, int64_t *dev_stats,
                            void *stream);
/* A bound on the read lengths of later _device batches (1..BWAGPU_MAX_READ_LEN,
   default BWAGPU_MAX_READ_LEN; the host entries take the exact maximum from
   seq_off).  The device sizes its LDS row buffers for it and launches only the
   length bins it reaches (a persistent grid over an empty bin still waits for
   the CU slots another stream's kernel holds).  A longer read sets
   dev_stats[3] bit 2 (as a read over BWAGPU_MAX_READ_LEN does) and gets no
   regions.  The per-read path (BWAGPU_C2A_PATH=fast) ignores it. */
int bwagpu_set_device_read_len(bwagpu_ctx_t *ctx, int32_t max_len);

int bwagpu_extend_batch(bwagpu_ctx_t *ctx, int32_t n_tasks, const bwagpu_ext_task_t *tasks,
                        const uint8_t *qpool, int64_t qpool_len, const uint8_t *tpool,
                        int64_t tpool_len, bwagpu_ext_result_t *results);

int bwagpu_align2_batch(bwagpu_ctx_t *ctx, int32_t n_tasks, const bwagpu_align2_task_t *tasks,
                        const uint8_t *qpool, int64_t qpool_len, const uint8_t *tpool, int64_t tpool_len,
                        bwagpu_kswr_t *results);
/* the same with tasks/pools/results in device memory; asynchronous on stream
   (hipStream_t, NULL = slot-0 stream).  dev_scratch: 8 x (sum of tlen + n_tasks)
   bytes of device memory for the row-maxima lists (ksw.c:191-198) */
int bwagpu_align2_device(bwagpu_ctx_t *ctx, int32_t n_tasks, const bwagpu_align2_task_t *dev_tasks,
                         const uint8_t *dev_qpool, const uint8_t *dev_tpool, bwagpu_kswr_t *dev_results,
                         void *dev_scratch, void *stream);

/* mem_reg2aln's CIGAR/NM/MD/position for n regions (host buffers; blocking).
   cigar: n * max_ops uint32, md: n * max_md bytes. */
int bwagpu_reg2aln_batch(bwagpu_ctx_t *ctx, int32_t n_tasks, const bwagpu_reg2aln_task_t *tasks,
                         const uint8_t *qpool, int64_t qpool_len, int32_t max_ops, int32_t max_md,
                         bwagpu_aln_t *out, uint32_t *cigar, char *md);

/* The FPGA wire format.  i_buf/i_words: one or more
   read records exactly as packReadData writes them (FPGAPipeline.cpp:252-336),
   back to back from word 0 (each record's first word is the word index of its
   end, relative to i_buf):
     end, l_seq, ceil(l_seq/8) words of 4-bit bases (first base in the high
     nibble), n_chains, then per chain: rmax[0], rmax[1] (int64, the window of
     getChainRef, FPGAPipeline.cpp:143-192), n_tasks, then per task: task index,
     rbeg (int64), qbeg, len.
   Every task is one seed extended left and right in its chain's window
   (bwamem.c:717-792: band retry, z-drop, local vs to-end); the record of task
   t is o_buf[10 t .. 10 t + 9] (int16): t & 0xffff, t >> 16, qb, qe - (qbeg +
   len), rb - rbeg, re - (rbeg + len), score, truesc, w, 0 — the fields
   processOutput applies (FPGAPipeline.cpp:91-105).  Task indices must be
   0..n-1, each once; *o_tasks = n.  o_cap_tasks bounds n.  A malformed
   stream returns BWAGPU_E_INVAL before any launch, or BWAGPU_E_RESULTS when
   the device finds it (a record that does not end at its end word, a task
   index out of range or repeated, a seed outside its window).  Reads up to
   BWAGPU_MAX_READ_LEN bp. */
int bwagpu_sw_stream(bwagpu_ctx_t *ctx, const int32_t *i_buf, int64_t i_words, int16_t *o_buf,
                     int32_t o_cap_tasks, int32_t *o_tasks);

int bwagpu_last_stats(const bwagpu_ctx_t *ctx, int slot, bwagpu_stats_t *stats);

/* Makes bwt the context's resident FM-index (copied to the device; a later
   call replaces it).  Replaces bwa's in-memory bwt_t for the seeding stage
   (bwa_idx_load_bwt, bwa/bwa.c:244-260; bwa-flow's SeqsToChains reads it through
   aux->idx->bwt, src/Pipeline.cpp:110-121). */
int bwagpu_set_bwt(bwagpu_ctx_t *ctx, const bwagpu_bwt_t *bwt);

/* mem_collect_intv (bwa/bwamem.c:120-167) for every read of a batch: the
   SMEMs (bwt_smem1, bwt.c:289-356), the re-seeding inside long SMEMs, the
   LAST-like pass (bwt_seed_strategy1, bwt.c:358-378), sorted by info as
   ks_introsort leaves them (bwamem.c:90-91, 166).  Reads: nt4 bases (0..4) at
   seq[seq_off[r]..seq_off[r+1]), host buffers, at most BWAGPU_MAX_SEED_READ
   bases.  out_n[r] = read r's interval count; the intervals of all reads go
   to out back to back in read order (read r's at sum(out_n[0..r))), at most
   out_cap of them.  max_per_read bounds one read's list on the device: a read
   with more gets out_n[r] = -(its count) and the call returns
   BWAGPU_E_UNSUPPORTED (out_n is still written); so does a batch whose total
   exceeds out_cap.  Blocking. */
int bwagpu_collect_intv(bwagpu_ctx_t *ctx, const bwagpu_seedopt_t *opt, int32_t n_reads, const int64_t *seq_off,
                        const uint8_t *seq, int32_t max_per_read, bwagpu_intv_t *out, int64_t out_cap,
                        int32_t *out_n);

/* bwt_sa (bwa/bwt.c:86-96) for n BWT positions k[i] in [0, seq_len]: out[i]
   = the forward-reverse coordinate mem_chain takes as a seed's rbeg
   (bwamem.c:288).  Needs the suffix array in bwagpu_set_bwt.  Blocking. */
int bwagpu_bwt_sa(bwagpu_ctx_t *ctx, int64_t n, const uint64_t *k, uint64_t *out);

/* ---- seeding's chaining: SeqsToChains on the device ---- */

/* a batch's chains in the bwagpu_batch_t layout: read r's chains are
   read_chain_off[r] .. read_chain_off[r+1]-1 (in the order bwa-flow's
   SeqsToChains leaves them), chain c's seeds chain_seed_off[c] ..
   chain_seed_off[c+1]-1 (mem_chain_t.seeds, in order) */
typedef struct {
  int32_t n_reads, n_chains;
  int64_t n_seeds;
  const int32_t *read_chain_off;  /* [n_reads+1]  */
  const int32_t *chain_seed_off;  /* [n_chains+1] */
  const bwagpu_chain_t *chains;   /* [n_chains]   */
  const bwagpu_seed_t *seeds;     /* [n_seeds]    */
} bwagpu_chains_t;

/* per-contig ALT flags (bntann1_t.is_alt, bwa/bntseq.h:41) that mem_chain
   copies into its chains and mem_chain_flt reads (bwamem.c:305, 359); n_seqs
   bytes, NULL = none (the default) */
int bwagpu_set_alt(bwagpu_ctx_t *ctx, const uint8_t *is_alt);

/* bwa-flow's SeqsToChains (src/bwa_wrapper.cpp:105-115) for every read of a
   batch: mem_collect_intv, then mem_chain's body (bwamem.c:260-330: bwt_sa of
   each interval's positions stepped to max_occ, bns_intv2rid, the kbtree of
   chains with test_and_merge), mem_chain_flt (336-396) and
   mem_flt_chained_seeds (607-624, mem_seed_sw through ksw_align2).  raw = 1
   stops after mem_chain (chains in kbtree order; w = kept = 0, first = -1).
   Reads as for bwagpu_collect_intv (host buffers, nt4, <= BWAGPU_MAX_SEED_READ
   bases); needs the suffix array in bwagpu_set_bwt.  *out points into
   context-owned pinned memory, valid until the next call on the context.
   Blocking. */
int bwagpu_seqs2chains(bwagpu_ctx_t *ctx, const bwagpu_seedopt_t *sopt, const bwagpu_chainopt_t *copt,
                       int32_t n_reads, const int64_t *seq_off, const uint8_t *seq, int32_t raw,
                       bwagpu_chains_t *out);

/* SeqsToChains and ChainsToRegions (src/Pipeline.cpp:110-121, 503-544) fused
   on the device: the chains never leave it.  out_n[r] = read r's regions
   (mem_chain2aln of each of its chains in order, as bwagpu_chain2aln returns
   them); *regs = every read's regions back to back in read order, *n_regs in
   all (context-owned pinned memory, valid until the next call).  Reads <=
   BWAGPU_MAX_READ_LEN.  BWAGPU_E_RESULTS as for bwagpu_chain2aln_wait.
   Blocking. */
int bwagpu_seqs2regions(bwagpu_ctx_t *ctx, const bwagpu_seedopt_t *sopt, const bwagpu_chainopt_t *copt,
                        int32_t n_reads, const int64_t *seq_off, const uint8_t *seq, int32_t *out_n,
                        const bwagpu_alnreg_t **regs, int64_t *n_regs);

/* Tuning, test and profiling entry points (bwagpu_debug_*, bwagpu_prof_*,
   bwagpu_ctx_ext_form / _row_bound, bwagpu_streams_concurrent) are declared
   in bwagpu_debug.h: none of them is part of the stage's interface, and the
   reference has no counterpart (it logs per-phase wall times instead,
   src/fpga/FPGAPipeline.cpp:557-578). */

#ifdef __cplusplus
}
#endif
#endif /* BWAGPU_H */
