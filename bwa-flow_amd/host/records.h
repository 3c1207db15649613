// records.h — the record types the SW stage consumes and produces, with the
// reference's memory layouts (so the stage links against bwa-flow's own
// objects unchanged).  Inside a bwa-flow build define BWAFLOW_NATIVE_HEADERS
// and the reference's headers are used instead of these mirrors.
//
//   bseq1_t        bwa/bwa.h:40-46 (bwa-flow flavour: + bams_t* bams)
//   mem_seed_t     src/bwa_wrapper.h:64-68            24 B
//   mem_chain_t    src/bwa_wrapper.h:70-77            40 B
//   mem_chain_v    src/bwa_wrapper.h:79-82
//   mem_alnreg_t   bwa/bwamem.h:60-79                 88 B
//   mem_alnreg_v   bwa/bwamem.h:80 (kvec: n, m, a)
//   ChainsRecord   src/Pipeline.h:46-57
//   RegionsRecord  src/Pipeline.h:59-65
#pragma once
#ifdef BWAFLOW_NATIVE_HEADERS
#include "Pipeline.h"
#include "bwa_wrapper.h"
#else
#include <stddef.h>
#include <stdint.h>

#include "bwagpu.h"

struct bams_t;
typedef struct {
  int l_seq, id;
  char *name, *comment, *seq, *qual, *sam;
  bams_t* bams;
} bseq1_t;

typedef struct {
  int64_t rbeg;
  int32_t qbeg, len;
  int score;
} mem_seed_t;

class mem_chain_t {
 public:
  int n, m, first, rid;
  uint32_t w : 29, kept : 2, is_alt : 1;
  float frac_rep;
  int64_t pos;
  mem_seed_t* seeds;
};

class mem_chain_v {
 public:
  size_t n, m;
  mem_chain_t* a;
};

typedef bwagpu_alnreg_t mem_alnreg_t;  // identical 88-byte layout (include/bwagpu.h)
typedef struct {
  size_t n, m;
  mem_alnreg_t* a;
} mem_alnreg_v;

struct bwtintv_t;
struct mem_chainref_t;

struct ChainsRecord {
  uint64_t start_idx;
  int batch_num;
  bseq1_t* seqs;
  mem_chain_v* chains;
  bwtintv_t** bwtintvs;
  size_t* bwtintv_nums;
  mem_alnreg_v* alnreg;
  mem_chainref_t** chain_ref;
  const char* name = "ChainsRecord";
  int tag;
};

struct RegionsRecord {
  uint64_t start_idx;
  int batch_num;
  bseq1_t* seqs;
  mem_chain_v* chains;
  mem_alnreg_v* alnreg;
  const char* name = "RegionsRecord";
};

static_assert(sizeof(mem_seed_t) == sizeof(bwagpu_seed_t), "mem_seed_t layout");
static_assert(sizeof(mem_chain_t) == 40, "mem_chain_t layout");
static_assert(sizeof(mem_alnreg_t) == 88, "mem_alnreg_t layout");
#endif
