/*
 * lzma_gpu.h -- C ABI of liblzmagpu.so, the MI355X (gfx950) LZMA decoder.
 *
 * Two surfaces:
 *
 *  1. Drop-in symbols of the reference decoder (LZMA SDK 9.20, the
 *     yurket/lzma-sdk-zlibLike fork).  Same names, argument meaning, enum
 *     values, struct layouts and SRes codes, so a caller linking the
 *     reference's LzmaDec.o / LzmaLib.o / Lzma2Dec.o can link this library
 *     instead.  Decoding runs on the GPU; only property parsing and
 *     allocation bookkeeping stay on the host.
 *
 *       LzmaProps_Decode        replaces LzmaDec.h:40  / LzmaDec.c:898-922
 *       LzmaDec_AllocateProbs   replaces LzmaDec.h:134 / LzmaDec.c:938-948
 *       LzmaDec_FreeProbs       replaces LzmaDec.h:135 / LzmaDec.c:880-884
 *       LzmaDec_Allocate        replaces LzmaDec.h:137 / LzmaDec.c:950-970
 *       LzmaDec_Free            replaces LzmaDec.h:138 / LzmaDec.c:892-896
 *       LzmaDec_Init            replaces LzmaDec.h:73  / LzmaDec.c:701-705
 *       LzmaDec_DecodeToDic     replaces LzmaDec.h:181-182 / LzmaDec.c:719-838
 *       LzmaDec_DecodeToBuf     replaces LzmaDec.h:198-199 / LzmaDec.c:840-878
 *       LzmaDecode              replaces LzmaDec.h:223-225 / LzmaDec.c:972-1002
 *       LzmaUncompress          replaces LzmaLib.h:128-129 / LzmaLib.c:41-46
 *       Lzma2Dec_AllocateProbs  replaces Lzma2Dec.h:31 / Lzma2Dec.c:75-80
 *       Lzma2Dec_Allocate       replaces Lzma2Dec.h:32 / Lzma2Dec.c:82-87
 *       Lzma2Dec_Init           replaces Lzma2Dec.h:33 / Lzma2Dec.c:89-96
 *       Lzma2Dec_DecodeToDic    replaces Lzma2Dec.h:51-52 / Lzma2Dec.c:170-289
 *       Lzma2Dec_DecodeToBuf    replaces Lzma2Dec.h:54-55 / Lzma2Dec.c:291-328
 *       Lzma2Decode             replaces Lzma2Dec.h:77-78 / Lzma2Dec.c:330-356
 *       LzmaDec_InitDicAndState exported like LzmaDec.c:685 (declared by Lzma2Dec.c:168)
 *
 *     Documented differences: no stdout print in LzmaDec_AllocateProbs (the
 *     fork's LzmaDec.c:945 debug printf); Lzma2Decode initialises its state
 *     (the reference one-call omits Lzma2Dec_Init, which is undefined
 *     behaviour); a dicLimit beyond dicBufSize returns SZ_ERROR_PARAM instead
 *     of writing out of bounds; after an LzmaDec_DecodeToDic / DecodeToBuf call
 *     that returns SZ_ERROR_DATA, dic[dicPos, ...) keeps its previous contents
 *     (the reference leaves the failed pass's partly decoded bytes there:
 *     LzmaDec.c:366-379 returns before the dicPos write-back at :413-423; the
 *     drop-in downloads only dic[old dicPos, new dicPos) -- both are bytes past
 *     dicPos, which the reference's contract never defines); without a usable
 *     HIP device every decode entry returns SZ_ERROR_FAIL and LzmaGpu_LastError()
 *     says why (there is no CPU fallback).
 *
 *  2. The batch extension (new): many independent streams per launch, all
 *     buffers caller-owned device memory, no allocation inside the call.
 */
#ifndef LZMA_GPU_H
#define LZMA_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- base ABI (Types.h:25-97,227-234) */

#ifndef SZ_OK
#define SZ_OK 0
#define SZ_ERROR_DATA 1
#define SZ_ERROR_MEM 2
#define SZ_ERROR_CRC 3
#define SZ_ERROR_UNSUPPORTED 4
#define SZ_ERROR_PARAM 5
#define SZ_ERROR_INPUT_EOF 6
#define SZ_ERROR_OUTPUT_EOF 7
#define SZ_ERROR_READ 8
#define SZ_ERROR_WRITE 9
#define SZ_ERROR_PROGRESS 10
#define SZ_ERROR_FAIL 11
#define SZ_ERROR_THREAD 12
#define SZ_ERROR_ARCHIVE 16
#define SZ_ERROR_NO_ARCHIVE 17
#endif

#ifndef __7Z_TYPES_H
typedef int SRes;
typedef unsigned char Byte;
typedef unsigned short UInt16;
typedef unsigned int UInt32;
typedef unsigned long long UInt64;
typedef size_t SizeT;
typedef int Bool;
typedef struct {
  void *(*Alloc)(void *p, size_t size);
  void (*Free)(void *p, void *address);
} ISzAlloc;
#endif

#define LZMA_PROPS_SIZE 5
#define LZMA_REQUIRED_INPUT_MAX 20

typedef UInt16 CLzmaProb; /* 16-bit probabilities (_LZMA_PROB32 not defined) */

typedef struct _CLzmaProps {
  unsigned lc, lp, pb;
  UInt32 dicSize;
} CLzmaProps;

/* Field order and types are the public layout of LzmaDec.h:50-69: callers of
 * the dictionary interface read dic/dicPos/dicBufSize directly. */
typedef struct {
  CLzmaProps prop;
  CLzmaProb *probs;
  Byte *dic;
  const Byte *buf;
  UInt32 range, code;
  SizeT dicPos;
  SizeT dicBufSize;
  UInt32 processedPos;
  UInt32 checkDicSize;
  unsigned state;
  UInt32 reps[4];
  unsigned remainLen;
  int needFlush;
  int needInitState;
  UInt32 numProbs;
  unsigned tempBufSize;
  Byte tempBuf[LZMA_REQUIRED_INPUT_MAX];
} CLzmaDec;

#define LzmaDec_Construct(p) { (p)->dic = 0; (p)->probs = 0; }

typedef enum { LZMA_FINISH_ANY, LZMA_FINISH_END } ELzmaFinishMode;

typedef enum {
  LZMA_STATUS_NOT_SPECIFIED,
  LZMA_STATUS_FINISHED_WITH_MARK,
  LZMA_STATUS_NOT_FINISHED,
  LZMA_STATUS_NEEDS_MORE_INPUT,
  LZMA_STATUS_MAYBE_FINISHED_WITHOUT_MARK
} ELzmaStatus;

/* ---------------------------------------------------------------- drop-in LzmaDec.h */

SRes LzmaProps_Decode(CLzmaProps *p, const Byte *data, unsigned size);
SRes LzmaDec_AllocateProbs(CLzmaDec *p, const Byte *props, unsigned propsSize, ISzAlloc *alloc);
void LzmaDec_FreeProbs(CLzmaDec *p, ISzAlloc *alloc);
SRes LzmaDec_Allocate(CLzmaDec *state, const Byte *prop, unsigned propsSize, ISzAlloc *alloc);
void LzmaDec_Free(CLzmaDec *state, ISzAlloc *alloc);
void LzmaDec_Init(CLzmaDec *p);
void LzmaDec_InitDicAndState(CLzmaDec *p, Bool initDic, Bool initState);
SRes LzmaDec_DecodeToDic(CLzmaDec *p, SizeT dicLimit, const Byte *src, SizeT *srcLen,
                         ELzmaFinishMode finishMode, ELzmaStatus *status);
SRes LzmaDec_DecodeToBuf(CLzmaDec *p, Byte *dest, SizeT *destLen, const Byte *src,
                         SizeT *srcLen, ELzmaFinishMode finishMode, ELzmaStatus *status);
SRes LzmaDecode(Byte *dest, SizeT *destLen, const Byte *src, SizeT *srcLen,
                const Byte *propData, unsigned propSize, ELzmaFinishMode finishMode,
                ELzmaStatus *status, ISzAlloc *alloc);

/* Device mirror of a decoder (dictionary interface).  LzmaDec_DecodeToDic /
 * LzmaDec_DecodeToBuf keep the decoder's dictionary, probability table and
 * state on the GPU between calls (keyed by the CLzmaDec address, its dic,
 * dicBufSize and probs allocation, and the current device): a call uploads
 * its input only -- plus, once per mirror, the dictionary history a
 * continuing decoder needs -- and downloads the bytes it decoded, the state
 * and the table.  Bytes of dic the CALLER writes between calls are seen when
 * it moves dicPos / processedPos over them as the reference's LZMA2 walker
 * does (Lzma2Dec.c:159-166: the call uploads exactly that span); any other
 * change of the positions, or of the host table, makes the call start from
 * the host copies.  A caller rewriting bytes it already handed to the decoder
 * without moving the positions is not detected: LzmaGpu_DecoderRelease(p)
 * drops the mirror (as do LzmaDec_FreeProbs / LzmaDec_Free and any change of
 * dic, dicBufSize or probs), so the next call starts from the host copy.  A
 * decoder used on another device drops its mirrors on the others.  Mirrors
 * beyond 256 decoders or 16 GiB (LZGPU_MIRROR_BUDGET_MB) are evicted least
 * recently used first. */
void LzmaGpu_DecoderRelease(const CLzmaDec *p);
/* Host<->device bytes moved by the drop-in decode entry points (LzmaDecode,
 * LzmaUncompress, Lzma2Decode, LzmaDec_DecodeToDic / DecodeToBuf and the LZMA2
 * streaming calls built on them) since start or the last reset, and the number
 * of decode calls that reached the device; reset != 0 zeroes them.  Any
 * argument may be NULL.  Process-wide. */
void LzmaGpu_DropinTransferStats(uint64_t *h2d_bytes, uint64_t *d2h_bytes, uint64_t *calls,
                                 int reset);
/* Coalesced calls (round 4): LzmaDecode / LzmaUncompress / Lzma2Decode calls
 * made by several host threads at once share batch launches, and so do
 * LzmaDec_DecodeToDic / LzmaDec_DecodeToBuf calls on different decoders (one
 * launch of the session kernels, one wave per decoder) -- group commit per
 * device: calls arriving while a launch runs form the next one; a lone
 * caller's launch has one item.  Counts since start or the last reset, summed
 * over devices and both kinds: launches, calls they carried, the largest
 * launch.  LZGPU_COALESCE=0 gives every call its own launch.  Any argument may
 * be NULL. */
void LzmaGpu_CoalesceStats(uint64_t *batches, uint64_t *calls, uint64_t *max_batch, int reset);
/* Host nanoseconds the one-call batches (LzmaDecode, LzmaUncompress,
 * Lzma2Decode) spent per phase, summed over batches since the last reset:
 * ns[0] plan, [1] staging (buffers, packing), [2] upload enqueue, [3] launch
 * enqueue, [4] waiting for the kernel and the results, [5] output download,
 * [6] whole batches, [7] every call from entry to return (queueing included);
 * *batches = batches timed.  Either pointer may be NULL. */
#define LZMA_GPU_COALESCE_PHASES 8
void LzmaGpu_CoalesceTimes(uint64_t *ns, uint64_t *batches, int reset);

/* ---------------------------------------------------------------- drop-in LzmaLib.h */

int LzmaUncompress(unsigned char *dest, size_t *destLen, const unsigned char *src,
                   SizeT *srcLen, const unsigned char *props, size_t propsSize);

/* ---------------------------------------------------------------- drop-in Lzma2Dec.h */

typedef struct {
  CLzmaDec decoder;
  UInt32 packSize;
  UInt32 unpackSize;
  int state;
  Byte control;
  Bool needInitDic;
  Bool needInitState;
  Bool needInitProp;
} CLzma2Dec;

#define Lzma2Dec_Construct(p) LzmaDec_Construct(&(p)->decoder)
#define Lzma2Dec_FreeProbs(p, alloc) LzmaDec_FreeProbs(&(p)->decoder, alloc);
#define Lzma2Dec_Free(p, alloc) LzmaDec_Free(&(p)->decoder, alloc);

SRes Lzma2Dec_AllocateProbs(CLzma2Dec *p, Byte prop, ISzAlloc *alloc);
SRes Lzma2Dec_Allocate(CLzma2Dec *p, Byte prop, ISzAlloc *alloc);
void Lzma2Dec_Init(CLzma2Dec *p);
SRes Lzma2Dec_DecodeToDic(CLzma2Dec *p, SizeT dicLimit, const Byte *src, SizeT *srcLen,
                          ELzmaFinishMode finishMode, ELzmaStatus *status);
SRes Lzma2Dec_DecodeToBuf(CLzma2Dec *p, Byte *dest, SizeT *destLen, const Byte *src,
                          SizeT *srcLen, ELzmaFinishMode finishMode, ELzmaStatus *status);
SRes Lzma2Decode(Byte *dest, SizeT *destLen, const Byte *src, SizeT *srcLen, Byte prop,
                 ELzmaFinishMode finishMode, ELzmaStatus *status, ISzAlloc *alloc);

/* ---------------------------------------------------------------- batch extension */

#define LZMA_GPU_KIND_LZMA 0  /* .lzma-style stream: props[0..5) = 5-byte header */
#define LZMA_GPU_KIND_LZMA2 1 /* LZMA2 byte range: props[0] = dictionary prop byte */
#define LZMA_GPU_NO_WORKSPACE (~(uint64_t)0)

/* One stream of a batch (48 bytes).  Offsets index the caller's packed
 * device buffers. probs_off is filled by LzmaGpu_PlanBatch. */
typedef struct LzmaGpuStreamDesc {
  uint64_t src_off;   /* compressed bytes start in d_src */
  uint64_t src_len;   /* compressed bytes available (*srcLen in) */
  uint64_t dst_off;   /* output window start in d_dst (window == dictionary) */
  uint64_t dst_cap;   /* output capacity (*destLen in) */
  uint64_t probs_off; /* in CLzmaProb cells, into the workspace */
  uint8_t props[5];
  uint8_t props_size;  /* propSize argument of LzmaDecode, normally 5 */
  uint8_t finish_mode; /* ELzmaFinishMode */
  uint8_t kind;        /* LZMA_GPU_KIND_* */
} LzmaGpuStreamDesc;

/* Per-stream outcome (24 bytes): exactly LzmaDecode's return value, *status
 * (-1 where LzmaDecode leaves it untouched), *destLen and *srcLen. */
typedef struct LzmaGpuResult {
  int32_t res;
  int32_t status;
  uint64_t dest_len;
  uint64_t src_len;
} LzmaGpuResult;

/* Host-side planner.  Fills descs[i].probs_off (16-byte aligned slices) and,
 * if order != NULL, a lane->stream permutation that groups streams of equal
 * table width and similar length into the same wavefront.  Returns the
 * workspace size in bytes (0 for n == 0). */
size_t LzmaGpu_PlanBatch(LzmaGpuStreamDesc *descs, size_t n, uint32_t *order);

/* Launch plan for LzmaGpu_DecodeBatchEx (filled by LzmaGpu_PlanBatchEx).
 * The lane order is partitioned: order[0, n_lds) runs on the LDS kernel in
 * n_classes launches by table width (class k: classes[k].n consecutive lanes,
 * per-stream probability tables in LDS, lanes_per_group streams per
 * workgroup); order[n_lds, n) runs on the generic kernel (tables in the
 * global workspace: lc + lp too wide for LDS).  Per-call overrides:
 * LzmaGpu_PlanBatchOpt.  PlanBatchEx reads experiment overrides from the
 * environment on every call: LZGPU_KERNEL=global|throughput|latency|coop,
 * LZGPU_LANES=<streams per workgroup>, LZGPU_GROUPS=<workgroups per CU>,
 * LZGPU_OCC=<1|2|4 waves per SIMD>, LZGPU_CUS, LZGPU_COOP=0|1,
 * LZGPU_PERSIST=0 (one stream per lane), LZGPU_CLASSES=1 (one LDS launch),
 * LZGPU_SLICE_ALIGN8=1, LZGPU_KERNEL_LZMA2=1, LZGPU_COOP_LAT=1, LZGPU_MERGE_LAT=0, LZGPU_ILV=0,
 * LZGPU_ILV_ANY=1, LZGPU_THR_FIT=0 (the
 * LZMA_GPU_PLAN_* flags below); DecodeBatchEx reads LZGPU_CLASS_STREAMS=0
 * (classes launched one after another on the caller's stream).
 * workspace_bytes includes the LDS launches' work counters at queue_offset
 * (zeroed by every DecodeBatchEx launch on its stream). */
#define LZMA_GPU_MAX_CLASSES 4
/* One LDS-kernel launch: `n` consecutive lanes of the order, tables of at most
 * lds_cells_per_lane cells, lanes_per_group streams per workgroup,
 * groups_per_cu workgroups per CU, register budget waves_per_simd. */
typedef struct LzmaGpuLdsClass {
  uint64_t n;
  uint32_t lanes_per_group;
  uint32_t lds_cells_per_lane;
  uint32_t groups_per_cu;
  uint32_t waves_per_simd;
  uint32_t lds_mask;      /* which probability sections live in LDS */
  uint32_t flags;         /* LZMA_GPU_CLASS_*: set by the planner */
  /* lane-interleaved global sections (lds_mask bit 30; the throughput
   * placement's default, LZMA_GPU_PLAN_NO_ILV turns it off): the class's slot
   * area in the workspace, in 16-bit cells -- slot_groups workgroups, each lane
   * group of 32 owning slot_cells rows of 32 cells; its streams get no
   * per-stream slice (probs_off 0) */
  uint64_t slot_off;
  uint32_t slot_cells;
  uint32_t slot_groups;
} LzmaGpuLdsClass;
/* the class holds LZMA2 items: launched on the kernel build with the LZMA2 chunk
 * walker (without it the LZMA-only build runs, fewer registers) */
#define LZMA_GPU_CLASS_HAS_LZMA2 1u

typedef struct LzmaGpuPlan {
  uint64_t workspace_bytes;
  uint64_t n;
  uint64_t n_lds;           /* lanes on the LDS kernel: sum of classes[k].n */
  uint32_t lanes_per_group; /* the class with the most streams (summary) */
  uint32_t lds_cells_per_lane;
  uint32_t groups_per_cu;
  uint32_t waves_per_simd;
  uint64_t queue_offset;    /* class k's work counter at queue_offset + 64 k */
  uint32_t persistent;      /* 1: grid = resident workgroups, lanes pull streams from the queue */
  uint32_t n_classes;       /* LDS launches, by table width (mixed lc/lp/pb batches) */
  LzmaGpuLdsClass classes[LZMA_GPU_MAX_CLASSES];
} LzmaGpuPlan;

SRes LzmaGpu_PlanBatchEx(LzmaGpuStreamDesc *descs, size_t n, uint32_t *order, LzmaGpuPlan *plan);

/* Per-call planner options (LzmaGpu_PlanBatchOpt).  Zero = the planner's own
 * choice for every field; the environment is not read.  `kernel` forces the
 * instantiation every LDS-eligible class runs on:
 *   THROUGHPUT  placement 0x105 (per-symbol tables in LDS), up to 32 streams
 *               per wave -- the config-3 kernel, whatever the batch size;
 *   LATENCY     placement 0x1BF, one stream per wave (lanes_per_group may
 *               widen it);
 *   COOP        one stream per 32-lane wave, every lane holding the
 *               stream's state (match copies and direct distance bits
 *               spread over the lanes); placement 0x7FF (all sections in
 *               LDS) where the whole table fits, else 0x1BF;
 *   GLOBAL      every stream on the generic kernel (tables in global memory).
 * A class whose latency-placement table exceeds the LDS limit keeps the
 * throughput placement.  cus: CUs to size the plan for (0 = the device's). */
#define LZMA_GPU_KERNEL_AUTO 0
#define LZMA_GPU_KERNEL_THROUGHPUT 1
#define LZMA_GPU_KERNEL_LATENCY 2
#define LZMA_GPU_KERNEL_COOP 3
#define LZMA_GPU_KERNEL_GLOBAL 4
typedef struct LzmaGpuPlanOptions {
  uint32_t kernel;          /* LZMA_GPU_KERNEL_* */
  uint32_t cus;             /* 0 = current device's CU count (256 without a device) */
  uint32_t lanes_per_group; /* 0 = planner; else streams per workgroup (<= 64) */
  uint32_t groups_per_cu;   /* 0 = planner */
  uint32_t waves_per_simd;  /* 0 = planner; else register budget 1|2|4 */
  uint32_t persistent;      /* 0 = default (on), 1 = on, 2 = off (one stream per lane) */
  uint32_t coop;            /* AUTO only: 0 = by streams per CU, 1 = always, 2 = never */
  uint32_t one_class;       /* 1: all LDS-eligible streams in one launch */
  uint32_t flags;           /* LZMA_GPU_PLAN_* bits */
  /* reserved, 0 (round 4's scalar-register share of one-lane waves, measured
   * slower at every share and removed in round 5) */
  uint32_t reserved;
} LzmaGpuPlanOptions;
/* per-lane LDS slices 8-byte aligned (default: an odd number of dwords, so that
 * 32 lanes reading the same cell index hit 32 different LDS banks) */
#define LZMA_GPU_PLAN_SLICE_ALIGN8 1u
/* every class on the kernel build with the LZMA2 chunk walker (A/B only) */
#define LZMA_GPU_PLAN_KERNEL_LZMA2 2u
/* cooperative classes keep the latency placement 0x1BF (SpecPos, matched-
 * literal trees and LenHigh in global memory).  Default: every section in LDS
 * (placement 0x7FF) when the whole table fits the class's streams per CU --
 * config 4 2.85 -> 3.00 GB/s, the xz leg 2.52 -> 2.63 (profiles/r02_ab/). */
#define LZMA_GPU_PLAN_COOP_LAT 4u
/* one class per table-width bucket even when several land in the one-lane
 * latency regime (default: those are merged into one class, one launch) */
#define LZMA_GPU_PLAN_NO_MERGE_LAT 8u
/* throughput classes keep the probability sections that are not in LDS in
 * per-stream slices (the round-2 layout) instead of lane-interleaved -- cell i
 * of the 32 lanes of a lane group side by side -- in a slot area per class
 * (LZGPU_ILV=0) */
#define LZMA_GPU_PLAN_NO_ILV 16u
/* A/B: interleaved rows for throughput waves of any width up to 64 lanes, not
 * only whole 32-lane groups (LZGPU_ILV_ANY=1) */
#define LZMA_GPU_PLAN_ILV_ANY 32u
/* Default: a single-class batch of 17 to 63 streams per CU in the latency
 * regime (a strong-scaling share, e.g. 8,192 x 4 KiB on 256 CUs) runs waves
 * of 2-4 streams so that every stream is resident at once, instead of
 * one-stream waves in several rounds.  This flag restores the round-2 shape
 * (LZGPU_THR_FIT=0). */
#define LZMA_GPU_PLAN_NO_THR_FIT 64u

/* Default: a one-lane latency class with more streams per CU than its widest
 * slice lets resident (lc + lp = 4 at pb = 4 takes 9 of a CU's 128 LDS blocks:
 * 14 workgroups) keeps its slot trees in the global rows instead, 8 blocks and
 * 16 workgroups per CU.  This flag keeps them in LDS (LZGPU_SLOTG=0). */
#define LZMA_GPU_PLAN_NO_SLOTG 256u
/* 128u was LZMA_GPU_PLAN_STEP (round 4's decision-level kernel, removed in
 * round 5): reserved, rejected with SZ_ERROR_PARAM so that a caller built
 * against the old header is told rather than silently given another flag. */
#define LZMA_GPU_PLAN_KNOWN_FLAGS 0x17Fu

/* LzmaGpu_PlanBatchEx with explicit options (opt == NULL: as PlanBatchEx,
 * whose defaults take the LZGPU_* experiment variables of the environment,
 * read per call).  SZ_ERROR_PARAM on an unknown kernel value or a flag bit
 * outside LZMA_GPU_PLAN_KNOWN_FLAGS. */
SRes LzmaGpu_PlanBatchOpt(LzmaGpuStreamDesc *descs, size_t n, uint32_t *order, LzmaGpuPlan *plan,
                          const LzmaGpuPlanOptions *opt);

/* Decode a planned batch (order is required: the plan's lane partition). */
SRes LzmaGpu_DecodeBatchEx(const LzmaGpuPlan *plan, const LzmaGpuStreamDesc *d_descs,
                           const uint32_t *d_order, const Byte *d_src, Byte *d_dst,
                           void *d_workspace, LzmaGpuResult *d_results, void *stream);

/* Decode n streams on the current HIP device (generic kernel, any plan).  All pointers are device
 * memory owned by the caller; d_order may be NULL (identity).  Asynchronous
 * on `stream` (a hipStream_t; NULL = default stream).  Returns SZ_OK if the
 * launch was queued; per-stream outcomes land in d_results. */
SRes LzmaGpu_DecodeBatch(const LzmaGpuStreamDesc *d_descs, const uint32_t *d_order, size_t n,
                         const Byte *d_src, Byte *d_dst, void *d_workspace,
                         size_t workspace_bytes, LzmaGpuResult *d_results, void *stream);

/* Convenience: the same over host buffers (allocates, copies, decodes,
 * copies back, frees).  descs need not be planned. */
SRes LzmaGpu_DecodeBatchHost(const LzmaGpuStreamDesc *descs, size_t n, const Byte *src,
                             size_t src_bytes, Byte *dst, size_t dst_bytes,
                             LzmaGpuResult *results);
/* The same with planner options (NULL = PlanBatchEx defaults); the plan used
 * is returned through plan_out when given. */
SRes LzmaGpu_DecodeBatchHostOpt(const LzmaGpuStreamDesc *descs, size_t n, const Byte *src,
                                size_t src_bytes, Byte *dst, size_t dst_bytes,
                                LzmaGpuResult *results, const LzmaGpuPlanOptions *opt,
                                LzmaGpuPlan *plan_out);

/* Split an LZMA2 stream into its independently decodable blocks: a block
 * starts at every chunk that resets the dictionary (control 0x01 or
 * >= 0xE0, Lzma2Dec.c:14-26) and runs to the next one.  Walks chunk headers
 * only (O(#chunks)).  For block i: src_off/src_len = its byte range
 * (the final EOS byte belongs to no block), unpack = its decoded size.
 * Returns the number of blocks (may exceed max_blocks: then only the first
 * max_blocks are written) or (size_t)-1 on a malformed header sequence. */
size_t Lzma2Gpu_SplitBlocks(const Byte *src, size_t src_len, uint64_t *src_off,
                            uint64_t *block_src_len, uint64_t *unpack, size_t max_blocks);

/* ---------------------------------------------------------------- streaming sessions */

/* A device-resident decoder: the CLzmaDec state (LzmaDec.h:50-69) plus one
 * call's arguments and results.  Many concurrent zlib-like streams (the fork's
 * SzDecodeLzmaToFileWithBuf pattern, 7zDec.c:567-648) advance by one batched
 * launch per round of calls; the state stays in device memory between calls.
 * All pointers are device memory. */
typedef struct LzmaGpuSession {
  uint32_t lc, lp, pb, dict_size;          /* CLzmaProps */
  uint16_t *probs;                         /* LzmaGpu_SessionProbsBytes() bytes */
  Byte *dic;                               /* dictionary (a ring for DecodeToBuf) */
  const Byte *in;                          /* this call: input */
  uint64_t dic_buf_size, dic_pos, dic_limit, in_len, in_used;
  uint32_t range, code, processed_pos, check_dic_size, state;
  uint32_t reps[4];
  uint32_t remain_len, need_flush, need_init_state, temp_buf_size;
  int32_t finish_mode, res, status;        /* this call: finish mode; results */
  int32_t mode;                            /* 0: DecodeToDic(dic_limit), 1: DecodeToBuf */
  Byte temp_buf[LZMA_REQUIRED_INPUT_MAX];
  Byte _pad[4];
  Byte *out;                               /* DecodeToBuf: destination */
  uint64_t out_len;                        /* DecodeToBuf: in = room, out = bytes written */
} LzmaGpuSession;

/* Device bytes a session's probability table needs for these props (0 on bad props). */
size_t LzmaGpu_SessionProbsBytes(const Byte *props, unsigned propsSize);
/* Host-side LzmaDec_Allocate + LzmaDec_Init on a session struct (LzmaDec.c:950-970,
 * 685-705): parses props, binds the caller's device probs / dictionary
 * (dic_buf_size >= 1; LzmaDec_Allocate uses the props' dictionary size). */
SRes LzmaGpu_SessionInit(LzmaGpuSession *s, const Byte *props, unsigned propsSize,
                         uint16_t *d_probs, Byte *d_dic, size_t dic_buf_size);
/* One call per session, all in one launch: for mode 0 exactly
 * LzmaDec_DecodeToDic(s, dic_limit, in, &in_len -> in_used, finish_mode, &status),
 * for mode 1 exactly LzmaDec_DecodeToBuf(s, out, &out_len, in, &in_len -> in_used,
 * finish_mode, &status); res / status / in_used / out_len and the decoder state are
 * written back into each d_sessions[i].  Asynchronous on `stream`. */
SRes LzmaGpu_SessionDecodeBatch(LzmaGpuSession *d_sessions, size_t n, void *stream);

/* ---------------------------------------------------------------- time-sliced batches */

/* A batch of LZMA streams decoded in rounds.  Each round is one launch in
 * which every unfinished stream makes one LzmaDec_DecodeToDic call
 * (LzmaDec.c:719-838) on its device-resident decoder (an LzmaGpuSession in the
 * workspace) with dicLimit = dicPos + slice_bytes and LZMA_FINISH_ANY -- the
 * call that reaches dst_cap takes the stream's own finish mode -- and its
 * state is spilled back for the next round (the CLzmaDec checkpoint,
 * LzmaDec.h:50-69).  Streams that finish drop out; the next round deals the
 * unfinished ones over every CU again.  Results (output bytes and
 * LzmaGpuResult) equal LzmaGpu_DecodeBatchEx's, i.e. LzmaDecode's per stream.
 * A round's launch is bounded by slice_bytes of output per stream, so work of
 * other streams or tenants queued on the device waits at most one round
 * behind a long stream, and a caller can stop after any round and resume --
 * with one exception: a stream whose round hits SZ_ERROR_DATA is decoded
 * again from its start in that same round as one unbounded call (the
 * reference's results on corrupt input depend on where its calls start,
 * LzmaDec.c:797,826; sliced.hip), so one corrupt long stream can hold a round
 * for a whole stream's worth of decode.
 * LZMA items only (an LZMA2 item: SZ_ERROR_PARAM at plan time). */
#define LZMA_GPU_SLICED_AUTO 0u
#define LZMA_GPU_SLICED_LANE 1u   /* one stream per wave, its table staged in LDS per round */
#define LZMA_GPU_SLICED_COOP 2u   /* one stream per 32-lane wave (the wave-cooperative decoder) */
#define LZMA_GPU_SLICED_GLOBAL 3u /* one stream per lane, table in the workspace (any lc/lp) */
typedef struct LzmaGpuSlicedPlan {
  uint64_t workspace_bytes;
  uint64_t n;
  uint64_t slice_bytes;
  uint32_t rounds;          /* launches that take every stream to its end: ceil(max dst_cap / slice) */
  uint32_t kernel;          /* LZMA_GPU_SLICED_* that runs */
  uint32_t table_cells;     /* LDS cells staged per stream (the widest, <= 32768) */
  uint32_t groups_per_cu;   /* resident workgroups per CU (persistent grid) */
  uint32_t max_groups;      /* grid of every round launch */
  uint32_t lds_mask;        /* LANE: sections staged in LDS (0x7FF all; 0x200001BF the
                               latency kernel's, the others used in place) */
  uint64_t sess_off, list_off, ctr_off; /* workspace sections (bytes) */
  uint64_t n_inplace;       /* streams whose table is wider than the staged slot: decoded
                               in place by the global kernel each round */
} LzmaGpuSlicedPlan;
/* Plan a sliced batch: fills descs[i].probs_off (the stream's table, in cells
 * into the workspace, 16-byte aligned), order (if not NULL: longest work
 * first, uploaded by the caller as DecodeBatchSliced's d_order) and *plan.
 * kernel = LZMA_GPU_SLICED_*; AUTO picks COOP for at most 8 streams per CU,
 * else LANE, and GLOBAL when no table fits LDS; streams whose table does not
 * fit the LDS kernel's slot (over 64 KiB) run in place on the global kernel
 * in the same rounds (plan->n_inplace).  SZ_ERROR_PARAM: slice_bytes == 0,
 * an LZMA2 item, more than 2^24 rounds. */
SRes LzmaGpu_PlanSliced(LzmaGpuStreamDesc *descs, size_t n, uint64_t slice_bytes, unsigned kernel,
                        uint32_t *order, LzmaGpuSlicedPlan *plan);
/* Enqueue rounds [first_round, first_round + n_rounds) of a planned batch on
 * `stream` (n_rounds 0 = every remaining round).  first_round 0 also resets
 * the workspace's counters and spills every stream's initial state.  Device
 * pointers as for DecodeBatchEx; d_order may be NULL (identity). */
SRes LzmaGpu_DecodeBatchSliced(const LzmaGpuSlicedPlan *plan, const LzmaGpuStreamDesc *d_descs,
                               const uint32_t *d_order, const Byte *d_src, Byte *d_dst,
                               void *d_workspace, LzmaGpuResult *d_results, unsigned first_round,
                               unsigned n_rounds, void *stream);
/* Streams still unfinished when round `round` starts (round = plan->rounds:
 * after the last; 0 once every stream is done).  Synchronises `stream`. */
SRes LzmaGpu_SlicedActive(const LzmaGpuSlicedPlan *plan, const void *d_workspace, unsigned round,
                          size_t *active, void *stream);
/* Host-buffer form (uploads, every round, downloads); plan_out may be NULL. */
SRes LzmaGpu_DecodeBatchSlicedHost(const LzmaGpuStreamDesc *descs, size_t n, const Byte *src,
                                   size_t src_bytes, Byte *dst, size_t dst_bytes,
                                   LzmaGpuResult *results, uint64_t slice_bytes, unsigned kernel,
                                   LzmaGpuSlicedPlan *plan_out);

/* ---------------------------------------------------------------- CRC-32 */

/* Drop-ins for 7zCrc.h (poly 0xEDB88320, 7zCrc.c:7):
 *   CrcGenerateTable  replaces 7zCrc.h:14 / 7zCrc.c:56-80 (no-op: device tables are constants)
 *   CrcUpdate         replaces 7zCrc.h:20 / 7zCrc.c:44-47 (raw register, no final XOR)
 *   CrcCalc           replaces 7zCrc.h:21 / 7zCrc.c:49-52 (init and final XOR 0xFFFFFFFF)
 * Over host buffers (upload + the batch kernels).  They have no error
 * channel: without a device they print once to stderr and return 0. */
void CrcGenerateTable(void);
UInt32 CrcUpdate(UInt32 crc, const void *data, size_t size);
UInt32 CrcCalc(const void *data, size_t size);

/* Batch CRC: range i is d_data[off[i] .. off[i] + len[i]).  Ranges are cut into
 * 2048-byte chunks (aligned to the range end) that decode in parallel.
 * Plan on the host from per-range capacities (len[i] <= caps[i]):
 *   n_chunks = CrcGpu_PlanChunks(caps, n, NULL, NULL);
 *   CrcGpu_PlanChunks(caps, n, chunk_base, chunk_range);  // n and n_chunks entries
 * then upload chunk_base / chunk_range.  Returns (size_t)-1 if n_chunks
 * would exceed 2^32 - 1.  d_chunk_crc: n_chunks uint32 of device scratch. */
size_t CrcGpu_PlanChunks(const uint64_t *caps, size_t n, uint32_t *chunk_base,
                         uint32_t *chunk_range);
/* d_crc[i] = register after range i from `init`, XOR `xorout`
 * (CrcCalc: init = xorout = 0xFFFFFFFF; CrcUpdate(v, ...): init = v, xorout = 0).
 * All pointers device memory; asynchronous on `stream`. */
SRes CrcGpu_Batch(const Byte *d_data, const uint64_t *d_off, const uint64_t *d_len, size_t n,
                  const uint32_t *d_chunk_base, const uint32_t *d_chunk_range, size_t n_chunks,
                  uint32_t init, uint32_t xorout, uint32_t *d_chunk_crc, uint32_t *d_crc,
                  void *stream);
/* CrcCalc of every decoded stream of a batch, straight from the decode's device
 * buffers: d_crc[i] = CrcCalc(d_dst + descs[i].dst_off, results[i].dest_len)
 * (the 7z folder / file check after decode, 7zIn.c:1380, 1397).  Plan with
 * capacities = descs[i].dst_cap via LzmaGpu_Crc32Plan (host descs). */
size_t LzmaGpu_Crc32Plan(const LzmaGpuStreamDesc *descs, size_t n, uint32_t *chunk_base,
                         uint32_t *chunk_range);
SRes LzmaGpu_Crc32Batch(const LzmaGpuStreamDesc *d_descs, const LzmaGpuResult *d_results,
                        size_t n, const Byte *d_dst, const uint32_t *d_chunk_base,
                        const uint32_t *d_chunk_range, size_t n_chunks, uint32_t *d_chunk_crc,
                        uint32_t *d_crc, void *stream);

/* ---------------------------------------------------------------- xz, x86 BCJ, CRC-64 */

/* x86 BCJ converter, drop-in for Bra.h:58 / Bra86.c:11-85 (x86_Convert: the
 * branch-target filter of 7z and xz; encoding 0 = decode).  Runs on the GPU
 * over the caller's host buffer; returns the bytes processed (the last <= 4
 * are left for the next call), *state carried like the reference's.  No
 * error channel: without a device it prints once and returns 0. */
SizeT x86_Convert(Byte *data, SizeT size, UInt32 ip, UInt32 *state, int encoding);

/* Batch x86 BCJ over device ranges, one lane per range, in place:
 * d_data[off[i] .. off[i] + len[i]) converted with start ip[i] and state
 * d_state[i] (in/out); d_done[i] = bytes processed.  Asynchronous on stream. */
SRes BcjGpu_X86Batch(Byte *d_data, const uint64_t *d_off, const uint64_t *d_len,
                     const uint32_t *d_ip, uint32_t *d_state, uint64_t *d_done, size_t n,
                     int encoding, void *stream);

/* RISC branch converters, drop-ins for Bra.h:59-63 (Bra.c ARM_Convert :6,
 * ARMT_Convert :33, PPC_Convert :68, SPARC_Convert :99; BraIA64.c
 * IA64_Convert :14): the same in-place conversion of the caller's host buffer,
 * computed on the GPU; returns the bytes processed (0 without a device).
 * ARM/PPC/SPARC convert one lane per 4-byte word, IA64 one per 16-byte bundle,
 * ARMT one lane per buffer (its matches chain). */
SizeT ARM_Convert(Byte *data, SizeT size, UInt32 ip, int encoding);
SizeT ARMT_Convert(Byte *data, SizeT size, UInt32 ip, int encoding);
SizeT PPC_Convert(Byte *data, SizeT size, UInt32 ip, int encoding);
SizeT SPARC_Convert(Byte *data, SizeT size, UInt32 ip, int encoding);
SizeT IA64_Convert(Byte *data, SizeT size, UInt32 ip, int encoding);

/* Delta filter, drop-ins for Delta.h:13-15 (Delta.c:6 Delta_Init, :20
 * Delta_Encode, :42 Delta_Decode).  state: DELTA_STATE_SIZE (256) bytes,
 * delta in 1..256; data converted in place on the GPU, state carried. */
#define LZMA_GPU_DELTA_STATE_SIZE 256
void Delta_Init(Byte *state);
void Delta_Encode(Byte *state, unsigned delta, Byte *data, SizeT size);
void Delta_Decode(Byte *state, unsigned delta, Byte *data, SizeT size);

/* Batch forms over device ranges, in place, asynchronous on stream.
 * BraGpu_Batch: kind = the xz filter ID (5 PPC, 6 IA64, 7 ARM, 8 ARMT,
 * 9 SPARC; else SZ_ERROR_UNSUPPORTED); range i starts at ip[i];
 * d_done[i] = what the reference's Convert returns for it.
 * DeltaGpu_Batch: d_delta[i] in 1..256 (unchecked on the device), d_state:
 * n x 256 bytes, range i's state at d_state + 256 * i (in/out). */
SRes BraGpu_Batch(unsigned kind, Byte *d_data, const uint64_t *d_off, const uint64_t *d_len,
                  const uint32_t *d_ip, uint64_t *d_done, size_t n, int encoding, void *stream);
SRes DeltaGpu_Batch(Byte *d_data, const uint64_t *d_off, const uint64_t *d_len,
                    const uint32_t *d_delta, Byte *d_state, size_t n, int encoding, void *stream);

/* BCJ2 (Bcj2.c:28-128), the four-stream x86 branch decoder of 7z: buf0 = main
 * stream, buf1 = CALL targets, buf2 = JMP / Jcc targets, buf3 = the range-coded
 * "converted" bits.  Bcj2_Decode replaces Bcj2.h:54-59 (host buffers, computed
 * on the GPU; buf0 may overlap outBuf as Bcj2.h:36-39 allows): SZ_OK or
 * SZ_ERROR_DATA as the reference, SZ_ERROR_FAIL without a device.
 * Bcj2Gpu_Batch: one lane per job, all pointers device memory, d_res[i] = the
 * SRes of job i; asynchronous on `stream`. */
typedef struct Bcj2GpuJob {   /* 80 bytes */
  const Byte *buf0, *buf1, *buf2, *buf3;
  uint64_t size0, size1, size2, size3;
  Byte *out;
  uint64_t out_size;
} Bcj2GpuJob;
int Bcj2_Decode(const Byte *buf0, SizeT size0, const Byte *buf1, SizeT size1, const Byte *buf2,
                SizeT size2, const Byte *buf3, SizeT size3, Byte *outBuf, SizeT outSize);
SRes Bcj2Gpu_Batch(const Bcj2GpuJob *d_jobs, size_t n, int32_t *d_res, void *stream);

/* CRC-64 (XzCrc64.c, poly 0xC96C5795D7870F42).  Crc64Calc drop-in replaces
 * XzCrc64.h:20 / XzCrc64.c:30 (host buffer, GPU compute; 0 without a device).
 * The batch form mirrors CrcGpu_Batch with 2048-byte chunks planned by
 * CrcGpu_PlanChunks; d_chunk_crc: n_chunks uint64 of scratch. */
UInt64 Crc64Calc(const void *data, size_t size);
SRes Crc64Gpu_Batch(const Byte *d_data, const uint64_t *d_off, const uint64_t *d_len, size_t n,
                    const uint32_t *d_chunk_base, const uint32_t *d_chunk_range, size_t n_chunks,
                    uint64_t init, uint64_t xorout, uint64_t *d_chunk_crc, uint64_t *d_crc,
                    void *stream);

/* xz files as block batches.  The reference decodes xz strictly in order
 * (XzUnpacker_Code, XzDec.c:604-870); the blocks of a multi-block file (and
 * the streams of a concatenated one) are independent, so here the whole file
 * is indexed first -- from each stream's footer and index backwards, as
 * Xzs_ReadBackward does (XzIn.c:150-280) -- and every block decodes as one
 * lane of an LZMA2 batch, then its filter chain (x86 / PPC / IA64 / ARM /
 * ARMT / SPARC branch converters, delta; last filter first, one batch per
 * kind and depth), then the block checks on the GPU (CRC-32, CRC-64;
 * SHA-256 on the host). */
#define LZMA_GPU_XZ_CHECK_NONE 0
#define LZMA_GPU_XZ_CHECK_CRC32 1
#define LZMA_GPU_XZ_CHECK_CRC64 4
#define LZMA_GPU_XZ_CHECK_SHA256 10
typedef struct {
  uint64_t header_off;  /* block header, offset in the file */
  uint64_t data_off;    /* first byte of the block's LZMA2 data */
  uint64_t pack_size;   /* LZMA2 data bytes (index unpadded size - header - check) */
  uint64_t unpack_size; /* uncompressed bytes (index) */
  uint64_t dst_off;     /* offset of the block's output in the whole file's output */
  uint64_t check_off;   /* stored check field, offset in the file */
  uint32_t check_type;  /* LZMA_GPU_XZ_CHECK_* of its stream */
  uint32_t check_size;  /* 0, 4, 8 or 32 bytes */
  uint32_t lzma2_prop;  /* dictionary byte of the LZMA2 filter (XZ_ID_LZMA2 0x21) */
  uint32_t x86;         /* 1: an x86 BCJ filter (XZ_ID_X86 4) precedes LZMA2 */
  uint32_t x86_ip;      /* its start offset (4-byte filter props, else 0) */
  uint32_t stream;      /* index of its xz stream in the file */
  uint32_t num_filters; /* filters before LZMA2 (0..3), in header order */
  uint32_t filter_id[3];   /* XZ_ID_Delta 3, X86 4, PPC 5, IA64 6, ARM 7, ARMT 8, SPARC 9 */
  uint32_t filter_prop[3]; /* start offset (branch converters) or distance 1..256 (delta) */
} LzmaGpuXzBlock;

/* Index an xz file (one or more concatenated streams with stream padding).
 * Fills up to `cap` blocks in file order, *n_blocks = the file's block count,
 * *unpack_total = the sum of their sizes.  Header, block-header, index and
 * footer validation follows XzDec.c / XzIn.c: SZ_ERROR_NO_ARCHIVE (magic or
 * stream-header CRC), SZ_ERROR_ARCHIVE (block header or index malformed),
 * SZ_ERROR_CRC (index CRC, index vs footer), SZ_ERROR_UNSUPPORTED (a filter
 * chain other than [x86 BCJ] + LZMA2, or stream flags beyond the check
 * field).  Host only: works without a device. */
SRes LzmaGpu_XzIndex(const Byte *file, size_t size, LzmaGpuXzBlock *blocks, size_t cap,
                     size_t *n_blocks, uint64_t *unpack_total);

/* Decode a whole xz file held in host memory: index, upload, one batch launch
 * over all blocks, BCJ, checks, download.  *destLen in: capacity, out: bytes
 * written (the whole output, or 0 on error).  Returns SZ_OK, an index error
 * above, SZ_ERROR_OUTPUT_EOF (capacity short), SZ_ERROR_DATA (a block's LZMA2
 * data does not decode to exactly its indexed size, ending with the end mark
 * in exactly its indexed bytes) or SZ_ERROR_CRC (a block check or non-zero
 * block padding).  *bad_block = the first failing block, or -1. */
SRes LzmaGpu_XzDecode(Byte *dest, SizeT *destLen, const Byte *file, size_t size,
                      int64_t *bad_block);

/* ---- 7z archives as folder batches ----------------
 * Replaces SzArEx_Open (7zIn.c:1314) + a SzArEx_Extract loop over every file
 * (7zIn.c:1322; ExtractAllFiles 7zIn.c:1405 in the fork): the header walk
 * runs on the host (an LZMA / LZMA2-packed header is decoded on the GPU),
 * every folder of the archive is one item of a single GPU batch, BCJ x86
 * and ARM folders go through the branch-converter kernels and every folder /
 * file CRC through one CRC-32 batch.  Folder shapes: Copy / LZMA / LZMA2,
 * optionally followed by BCJ x86 or ARM (CheckSupportedFolder, 7zDec.c:269;
 * ARM_Convert at ip 0, :449); BCJ2 folders, which the reference also
 * decodes, return SZ_ERROR_UNSUPPORTED here. */
typedef struct LzmaGpu7zFolder {   /* 80 bytes */
  uint64_t pack_off;     /* archive offset of the main coder's pack stream */
  uint64_t pack_size;
  uint64_t unpack_size;  /* SzFolder_GetUnpackSize */
  uint64_t dst_off;      /* offset of the folder's output in the extraction buffer */
  uint64_t method;       /* coder 0 method id (0 Copy, 0x030101 LZMA, 0x21 LZMA2) */
  uint32_t x86;          /* 1: a BCJ x86 coder follows */
  uint32_t supported;    /* SZ_OK, or the SRes the folder fails with before decoding */
  uint32_t crc_defined, crc;
  uint32_t first_file;   /* FolderStartFileIndex */
  uint32_t num_files;    /* NumUnpackStreams */
  uint32_t num_coders;
  uint32_t props_size;
  Byte props[8];
} LzmaGpu7zFolder;

typedef struct LzmaGpu7zFile {     /* 48 bytes */
  uint64_t size;
  uint64_t dst_off;      /* offset of the file's bytes in the extraction buffer */
  uint32_t folder;       /* FileIndexToFolderIndexMap: 0xFFFFFFFF = no data */
  uint32_t crc, crc_defined;
  uint32_t has_stream, is_dir;
  uint32_t name_off, name_len;  /* UTF-16 units into the names buffer (name_len counts the NUL) */
  uint32_t reserved;
} LzmaGpu7zFile;

/* SzArEx_Open: SZ_OK or its error (SZ_ERROR_NO_ARCHIVE, _UNSUPPORTED, _CRC,
 * _ARCHIVE, _INPUT_EOF, a packed header's decode error).  Fills up to
 * folder_cap / file_cap / names_cap entries (any pointer may be NULL); the
 * counts and *unpack_total (the extraction buffer size) are always set. */
SRes LzmaGpu_7zOpen(const Byte *archive, size_t size, LzmaGpu7zFolder *folders,
                    size_t folder_cap, size_t *n_folders, LzmaGpu7zFile *files, size_t file_cap,
                    size_t *n_files, UInt16 *names, size_t names_cap, size_t *names_len,
                    UInt64 *unpack_total);

/* Every folder decoded into dest (folders back to back, files at their
 * LzmaGpu7zFile.dst_off); *destLen in: capacity (SZ_ERROR_OUTPUT_EOF if
 * below unpack_total), out: unpack_total.  file_res[i] = what SzArEx_Extract
 * returns for file i with a fresh folder cache (SZ_OK, the folder's decode
 * error, SZ_ERROR_CRC, SZ_ERROR_FAIL).  Returns SzArEx_Open's error, else the
 * first file's non-OK result, else SZ_OK. */
SRes LzmaGpu_7zExtract(Byte *dest, SizeT *destLen, const Byte *archive, size_t size,
                       SRes *file_res, size_t file_cap);

/* Device / diagnostics. */
int LzmaGpu_DeviceCount(void);
const char *LzmaGpu_LastError(void);
const char *LzmaGpu_Version(void);

#ifdef __cplusplus
}
#endif

#endif /* LZMA_GPU_H */
