/*
 * lzma_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker, never shipped).
 *
 * A from-scratch CPU restatement of the reference decoder's *observable*
 * behaviour: output bytes plus {res, status, destLen, srcLen} for every
 * finish mode, truncation and corruption.  Observable behaviour depends on
 * the reference's internal call segmentation (bulk pass limited to
 * inSize-20, single-symbol tail passes after a dry-run look-ahead, the
 * dictionary-size split), so the driver functions follow the same
 * segmentation; the symbol decoder itself is written as plain functions.
 *
 * Reference map (file:line in /root/reference):
 *   range-coder bit / tree      LzmaDec.c:8-45         -> rc_bit, rc_tree
 *   direct bits                 LzmaDec.c:323-344      -> rc_direct
 *   symbol loop                 LzmaDec.c:131-426      -> orc_run
 *   pending-match flush         LzmaDec.c:428-452      -> orc_flush_pending
 *   dictionary-size split loop  LzmaDec.c:454-477      -> orc_run_split
 *   look-ahead dry run          LzmaDec.c:487-675      -> orc_probe
 *   rc init / state init        LzmaDec.c:678-717      -> orc_init_*
 *   DecodeToDic driver          LzmaDec.c:719-838      -> orc_decode_to_dic
 *   DecodeToBuf ring driver     LzmaDec.c:840-878      -> orc_decode_to_buf
 *   props                       LzmaDec.c:898-922      -> orc_props_parse
 *   LzmaDecode one-call         LzmaDec.c:972-1002     -> orc_lzma_decode
 *   LzmaUncompress              LzmaLib.c:41-46        -> orc_lzma_uncompress
 *   LZMA2 chunk parser/driver   Lzma2Dec.c:98-289      -> orc2_*
 */
#include "lzma_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

enum { RES_OK = 0, RES_DATA = 1, RES_MEM = 2, RES_UNSUPPORTED = 4, RES_INPUT_EOF = 6 };
enum { ST_NONE = 0, ST_DONE_MARK = 1, ST_NOT_DONE = 2, ST_MORE_INPUT = 3, ST_MAYBE_DONE = 4 };
enum { FIN_ANY = 0, FIN_END = 1 };

#define TOP_VALUE (1u << 24)
#define PROB_ONE 2048u
#define PROB_INIT 1024u
#define LOOKAHEAD_MAX 20u /* LZMA_REQUIRED_INPUT_MAX, LzmaDec.h:48 */
#define LEN_DONE 274u     /* 2 + 8 + 8 + 256: "stream finished" marker value */

/* Probability-table layout of the LZMA format (offsets in 16-bit cells). */
enum {
  P_IS_MATCH = 0,                 /* [12 states][16 posStates] */
  P_IS_REP = 192,                 /* [12] */
  P_IS_REP_G0 = 204,              /* [12] */
  P_IS_REP_G1 = 216,              /* [12] */
  P_IS_REP_G2 = 228,              /* [12] */
  P_IS_REP0_LONG = 240,           /* [12][16] */
  P_POS_SLOT = 432,               /* [4][64] */
  P_SPEC_POS = 688,               /* [114] */
  P_ALIGN = 802,                  /* [16] */
  P_LEN = 818,                    /* length coder, 514 cells */
  P_REP_LEN = 1332,               /* rep-length coder, 514 cells */
  P_LITERAL = 1846                /* [0x300 << (lc+lp)] */
};
/* inside a length coder */
enum { L_CHOICE = 0, L_CHOICE2 = 1, L_LOW = 2, L_MID = 130, L_HIGH = 258 };

typedef struct {
  unsigned lc, lp, pb;
  uint32_t dict_size;
} orc_props;

typedef struct {
  orc_props pr;
  uint16_t *probs;
  uint32_t nprobs;
  uint8_t *dic;
  size_t dic_cap;
  size_t dic_pos;
  const uint8_t *in;      /* read cursor of the current bulk pass */
  uint32_t range, code;
  uint32_t total;         /* processedPos */
  uint32_t full;          /* checkDicSize: 0 until dict_size bytes were produced */
  unsigned st;            /* LZMA state 0..11 */
  uint32_t rep[4];
  unsigned pending;       /* remainLen */
  int need_rc_init;       /* needFlush */
  int need_state_init;    /* needInitState */
  unsigned tmp_n;
  uint8_t tmp[LOOKAHEAD_MAX];
} orc_dec;

/* ---------------------------------------------------------------- props */

static int orc_props_parse(orc_props *p, const uint8_t *b, unsigned n) {
  uint32_t dict;
  unsigned d;
  if (n < 5) return RES_UNSUPPORTED;
  dict = (uint32_t)b[1] | ((uint32_t)b[2] << 8) | ((uint32_t)b[3] << 16) |
         ((uint32_t)b[4] << 24);
  if (dict < 4096) dict = 4096;
  p->dict_size = dict;
  d = b[0];
  if (d >= 225) return RES_UNSUPPORTED;
  p->lc = d % 9;
  p->lp = (d / 9) % 5;
  p->pb = d / 45;
  return RES_OK;
}

static uint32_t orc_num_probs(const orc_props *p) {
  return 1846u + (768u << (p->lc + p->lp));
}

/* ---------------------------------------------------------------- range coder */

typedef struct {
  uint32_t range, code;
  const uint8_t *in;
} rc_t;

static inline void rc_norm(rc_t *rc) {
  if (rc->range < TOP_VALUE) {
    rc->range <<= 8;
    rc->code = (rc->code << 8) | *rc->in++;
  }
}

/* One adaptive binary decision; updates *prob. */
static inline unsigned rc_bit(rc_t *rc, uint16_t *prob) {
  uint32_t p = *prob, bound;
  rc_norm(rc);
  bound = (rc->range >> 11) * p;
  if (rc->code < bound) {
    rc->range = bound;
    *prob = (uint16_t)(p + ((PROB_ONE - p) >> 5));
    return 0;
  }
  rc->range -= bound;
  rc->code -= bound;
  *prob = (uint16_t)(p - (p >> 5));
  return 1;
}

/* MSB-first bit tree of `bits` levels; returns symbol in [0, 1<<bits). */
static inline unsigned rc_tree(rc_t *rc, uint16_t *probs, unsigned bits) {
  unsigned m = 1, lim = 1u << bits;
  while (m < lim) m = (m << 1) | rc_bit(rc, probs + m);
  return m - lim;
}

/* One fixed-probability ("direct") bit appended to *v, exactly in the
 * reference's arithmetic form (LzmaDec.c:325-334). */
static inline void rc_direct(rc_t *rc, uint32_t *v) {
  uint32_t t;
  rc_norm(rc);
  rc->range >>= 1;
  rc->code -= rc->range;
  t = 0u - (rc->code >> 31);
  *v = (*v << 1) + (t + 1u);
  rc->code += rc->range & t;
}

static inline size_t ring_back(size_t pos, uint32_t dist, size_t cap) {
  return pos - dist + (pos < dist ? cap : 0);
}

/* ---------------------------------------------------------------- symbol loop */

/*
 * Decode symbols until dic_pos reaches `limit` or the read cursor reaches
 * `in_limit` (checked after each whole symbol; the first symbol is always
 * decoded).  Restates LzmaDec_DecodeReal (LzmaDec.c:131-426).
 * Returns 0 or RES_DATA.
 */
static int orc_run(orc_dec *d, size_t limit, const uint8_t *in_limit) {
  uint16_t *pr = d->probs;
  unsigned st = d->st;
  uint32_t r0 = d->rep[0], r1 = d->rep[1], r2 = d->rep[2], r3 = d->rep[3];
  const unsigned pb_mask = (1u << d->pr.pb) - 1, lp_mask = (1u << d->pr.lp) - 1;
  const unsigned lc = d->pr.lc;
  uint8_t *dic = d->dic;
  const size_t cap = d->dic_cap;
  size_t pos = d->dic_pos;
  uint32_t total = d->total, full = d->full;
  unsigned len = 0;
  rc_t rc;
  rc.range = d->range;
  rc.code = d->code;
  rc.in = d->in;

  do {
    const unsigned ps = total & pb_mask;
    unsigned lcoder;

    if (!rc_bit(&rc, pr + P_IS_MATCH + (st << 4) + ps)) {
      /* ---- literal (LzmaDec.c:161-196) */
      uint16_t *lit = pr + P_LITERAL;
      unsigned sym = 1;
      if (full != 0 || total != 0) {
        unsigned prev = dic[(pos == 0 ? cap : pos) - 1];
        lit += 768u * (((total & lp_mask) << lc) + (prev >> (8 - lc)));
      }
      if (st < 7) {
        st = (st < 4) ? 0 : st - 3;
        while (sym < 0x100) sym = (sym << 1) | rc_bit(&rc, lit + sym);
      } else {
        unsigned mbyte = dic[ring_back(pos, r0, cap)];
        unsigned offs = 0x100;
        st = (st < 10) ? st - 3 : st - 6;
        while (sym < 0x100) {
          unsigned mbit, b;
          mbyte <<= 1;
          mbit = mbyte & offs;
          b = rc_bit(&rc, lit + offs + mbit + sym);
          sym = (sym << 1) | b;
          offs = b ? (offs & mbit) : (offs & ~mbit);
        }
      }
      dic[pos++] = (uint8_t)sym;
      total++;
      continue;
    }

    if (!rc_bit(&rc, pr + P_IS_REP + st)) {
      /* ---- new match: distance follows the length */
      st += 12;
      lcoder = P_LEN;
    } else {
      /* ---- repeated match (LzmaDec.c:207-260) */
      if (full == 0 && total == 0) return RES_DATA;
      if (!rc_bit(&rc, pr + P_IS_REP_G0 + st)) {
        if (!rc_bit(&rc, pr + P_IS_REP0_LONG + (st << 4) + ps)) {
          /* short rep: one byte from rep0 */
          dic[pos] = dic[ring_back(pos, r0, cap)];
          pos++;
          total++;
          st = (st < 7) ? 9 : 11;
          continue;
        }
      } else {
        uint32_t dist;
        if (!rc_bit(&rc, pr + P_IS_REP_G1 + st)) {
          dist = r1;
        } else {
          if (!rc_bit(&rc, pr + P_IS_REP_G2 + st)) {
            dist = r2;
          } else {
            dist = r3;
            r3 = r2;
          }
          r2 = r1;
        }
        r1 = r0;
        r0 = dist;
      }
      st = (st < 7) ? 8 : 11;
      lcoder = P_REP_LEN;
    }

    /* ---- length (LzmaDec.c:261-292) */
    if (!rc_bit(&rc, pr + lcoder + L_CHOICE))
      len = rc_tree(&rc, pr + lcoder + L_LOW + (ps << 3), 3);
    else if (!rc_bit(&rc, pr + lcoder + L_CHOICE2))
      len = 8 + rc_tree(&rc, pr + lcoder + L_MID + (ps << 3), 3);
    else
      len = 16 + rc_tree(&rc, pr + lcoder + L_HIGH, 8);

    if (st >= 12) {
      /* ---- distance (LzmaDec.c:294-374) */
      unsigned lstate = len < 4 ? len : 3;
      uint32_t dist = rc_tree(&rc, pr + P_POS_SLOT + (lstate << 6), 6);
      if (dist >= 4) {
        const unsigned slot = dist;
        unsigned nbits = (slot >> 1) - 1;
        dist = 2 | (slot & 1);
        if (slot < 14) {
          /* reverse bit tree in SpecPos */
          uint16_t *sp;
          uint32_t mask = 1;
          unsigned node = 1;
          dist <<= nbits;
          sp = pr + P_SPEC_POS + dist - slot - 1;
          do {
            if (rc_bit(&rc, sp + node)) {
              node = (node << 1) | 1;
              dist |= mask;
            } else {
              node <<= 1;
            }
            mask <<= 1;
          } while (--nbits != 0);
        } else {
          unsigned node = 1, k;
          nbits -= 4;
          do rc_direct(&rc, &dist); while (--nbits != 0);
          dist <<= 4;
          for (k = 0; k < 4; k++) {
            unsigned b = rc_bit(&rc, pr + P_ALIGN + node);
            node = (node << 1) | b;
            dist |= (uint32_t)b << k;
          }
          if (dist == 0xFFFFFFFFu) {
            /* end-of-stream marker */
            len += LEN_DONE;
            st -= 12;
            break;
          }
        }
      }
      r3 = r2;
      r2 = r1;
      r1 = r0;
      r0 = dist + 1;
      if (full == 0) {
        if (dist >= total) return RES_DATA;
      } else if (dist >= full) {
        return RES_DATA;
      }
      st = (st < 19) ? 7 : 10;
    }

    /* ---- copy (LzmaDec.c:376-408), byte-serial overlap semantics */
    len += 2;
    if (limit == pos) return RES_DATA;
    {
      size_t room = limit - pos;
      unsigned n = (room < len) ? (unsigned)room : len;
      size_t from = ring_back(pos, r0, cap);
      total += n;
      len -= n;
      while (n-- != 0) {
        dic[pos++] = dic[from];
        if (++from == cap) from = 0;
      }
    }
  } while (pos < limit && rc.in < in_limit);

  rc_norm(&rc);
  d->in = rc.in;
  d->range = rc.range;
  d->code = rc.code;
  d->pending = len;
  d->dic_pos = pos;
  d->total = total;
  d->rep[0] = r0;
  d->rep[1] = r1;
  d->rep[2] = r2;
  d->rep[3] = r3;
  d->st = st;
  return RES_OK;
}

/* Finish a match that a previous pass clipped at its output limit
 * (LzmaDec.c:428-452). */
static void orc_flush_pending(orc_dec *d, size_t limit) {
  unsigned n;
  if (d->pending == 0 || d->pending >= LEN_DONE) return;
  n = d->pending;
  if (limit - d->dic_pos < n) n = (unsigned)(limit - d->dic_pos);
  if (d->full == 0 && d->pr.dict_size - d->total <= n) d->full = d->pr.dict_size;
  d->total += n;
  d->pending -= n;
  while (n-- != 0) {
    d->dic[d->dic_pos] = d->dic[ring_back(d->dic_pos, d->rep[0], d->dic_cap)];
    d->dic_pos++;
  }
}

/* Bulk decode, splitting passes exactly where total reaches dict_size so
 * `full` switches on there (LzmaDec.c:454-477). */
static int orc_run_split(orc_dec *d, size_t limit, const uint8_t *in_limit) {
  do {
    size_t lim = limit;
    if (d->full == 0) {
      uint32_t left = d->pr.dict_size - d->total;
      if (limit - d->dic_pos > left) lim = d->dic_pos + left;
    }
    if (orc_run(d, lim, in_limit) != RES_OK) return RES_DATA;
    if (d->total >= d->pr.dict_size) d->full = d->pr.dict_size;
    orc_flush_pending(d, limit);
  } while (d->dic_pos < limit && d->in < in_limit && d->pending < LEN_DONE);
  if (d->pending > LEN_DONE) d->pending = LEN_DONE;
  return RES_OK;
}

/* ---------------------------------------------------------------- dry run */

enum { PROBE_SHORT = 0, PROBE_LIT = 1, PROBE_MATCH = 2, PROBE_REP = 3 };

typedef struct {
  uint32_t range, code;
  const uint8_t *in, *end;
  int short_input;
} probe_t;

static inline int pr_norm(probe_t *t) {
  if (t->range < TOP_VALUE) {
    if (t->in >= t->end) { t->short_input = 1; return 0; }
    t->range <<= 8;
    t->code = (t->code << 8) | *t->in++;
  }
  return 1;
}

/* Decision without adapting the probability; returns 0/1, or -1 if the
 * input ran out. */
static inline int pr_bit(probe_t *t, const uint16_t *prob) {
  uint32_t bound;
  if (!pr_norm(t)) return -1;
  bound = (t->range >> 11) * *prob;
  if (t->code < bound) { t->range = bound; return 0; }
  t->range -= bound;
  t->code -= bound;
  return 1;
}

static inline int pr_tree(probe_t *t, const uint16_t *probs, unsigned bits, unsigned *out) {
  unsigned m = 1, lim = 1u << bits;
  while (m < lim) {
    int b = pr_bit(t, probs + m);
    if (b < 0) return 0;
    m = (m << 1) | (unsigned)b;
  }
  *out = m - lim;
  return 1;
}

/*
 * Would one more symbol decode from [in, in+n) without running out of input?
 * Restates LzmaDec_TryDummy (LzmaDec.c:487-675): no state or probability is
 * modified; returns PROBE_SHORT if the input is too short, else the kind of
 * symbol found.
 */
static int orc_probe(const orc_dec *d, const uint8_t *in, size_t n) {
  const uint16_t *pr = d->probs;
  const unsigned ps = d->total & ((1u << d->pr.pb) - 1);
  unsigned st = d->st;
  int kind, b;
  unsigned lcoder, len = 0;
  probe_t t;
  t.range = d->range;
  t.code = d->code;
  t.in = in;
  t.end = in + n;
  t.short_input = 0;

#define PB(prob) do { b = pr_bit(&t, (prob)); if (b < 0) return PROBE_SHORT; } while (0)

  PB(pr + P_IS_MATCH + (st << 4) + ps);
  if (b == 0) {
    const uint16_t *lit = pr + P_LITERAL;
    unsigned sym = 1;
    if (d->full != 0 || d->total != 0) {
      unsigned prev = d->dic[(d->dic_pos == 0 ? d->dic_cap : d->dic_pos) - 1];
      lit += 768u * (((d->total & ((1u << d->pr.lp) - 1)) << d->pr.lc) +
                     (prev >> (8 - d->pr.lc)));
    }
    if (st < 7) {
      while (sym < 0x100) {
        PB(lit + sym);
        sym = (sym << 1) | (unsigned)b;
      }
    } else {
      unsigned mbyte = d->dic[ring_back(d->dic_pos, d->rep[0], d->dic_cap)];
      unsigned offs = 0x100;
      while (sym < 0x100) {
        unsigned mbit;
        mbyte <<= 1;
        mbit = mbyte & offs;
        PB(lit + offs + mbit + sym);
        sym = (sym << 1) | (unsigned)b;
        offs = b ? (offs & mbit) : (offs & ~mbit);
      }
    }
    kind = PROBE_LIT;
  } else {
    PB(pr + P_IS_REP + st);
    if (b == 0) {
      st = 0; /* marks "distance follows" */
      lcoder = P_LEN;
      kind = PROBE_MATCH;
    } else {
      kind = PROBE_REP;
      PB(pr + P_IS_REP_G0 + st);
      if (b == 0) {
        PB(pr + P_IS_REP0_LONG + (st << 4) + ps);
        if (b == 0) {
          if (!pr_norm(&t)) return PROBE_SHORT;
          return PROBE_REP;
        }
      } else {
        PB(pr + P_IS_REP_G1 + st);
        if (b != 0) PB(pr + P_IS_REP_G2 + st);
      }
      st = 12;
      lcoder = P_REP_LEN;
    }
    PB(pr + lcoder + L_CHOICE);
    if (b == 0) {
      if (!pr_tree(&t, pr + lcoder + L_LOW + (ps << 3), 3, &len)) return PROBE_SHORT;
    } else {
      PB(pr + lcoder + L_CHOICE2);
      if (b == 0) {
        if (!pr_tree(&t, pr + lcoder + L_MID + (ps << 3), 3, &len)) return PROBE_SHORT;
        len += 8;
      } else {
        if (!pr_tree(&t, pr + lcoder + L_HIGH, 8, &len)) return PROBE_SHORT;
        len += 16;
      }
    }
    if (st < 4) {
      unsigned slot;
      if (!pr_tree(&t, pr + P_POS_SLOT + ((len < 4 ? len : 3) << 6), 6, &slot))
        return PROBE_SHORT;
      if (slot >= 4) {
        unsigned nbits = (slot >> 1) - 1, node = 1;
        const uint16_t *base;
        if (slot < 14) {
          base = pr + P_SPEC_POS + ((2u | (slot & 1)) << nbits) - slot - 1;
        } else {
          nbits -= 4;
          do {
            if (!pr_norm(&t)) return PROBE_SHORT;
            t.range >>= 1;
            t.code -= t.range & (((t.code - t.range) >> 31) - 1);
          } while (--nbits != 0);
          base = pr + P_ALIGN;
          nbits = 4;
        }
        do {
          PB(base + node);
          node = (node << 1) | (unsigned)b;
        } while (--nbits != 0);
      }
    }
  }
#undef PB
  if (!pr_norm(&t)) return PROBE_SHORT;
  return kind;
}

/* ---------------------------------------------------------------- init */

static void orc_init_state_real(orc_dec *d) {
  uint32_t i, n = orc_num_probs(&d->pr);
  for (i = 0; i < n; i++) d->probs[i] = PROB_INIT;
  d->rep[0] = d->rep[1] = d->rep[2] = d->rep[3] = 1;
  d->st = 0;
  d->need_state_init = 0;
}

static void orc_init_dic_state(orc_dec *d, int init_dic, int init_state) {
  d->need_rc_init = 1;
  d->pending = 0;
  d->tmp_n = 0;
  if (init_dic) {
    d->total = 0;
    d->full = 0;
    d->need_state_init = 1;
  }
  if (init_state) d->need_state_init = 1;
}

static void orc_init(orc_dec *d) {
  d->dic_pos = 0;
  orc_init_dic_state(d, 1, 1);
}

/* ---------------------------------------------------------------- drivers */

/* LzmaDec_DecodeToDic (LzmaDec.c:719-838). */
static int orc_decode_to_dic(orc_dec *d, size_t dic_limit, const uint8_t *src,
                             size_t *src_len, int fin, int *status) {
  size_t avail = *src_len;
  *src_len = 0;
  orc_flush_pending(d, dic_limit);
  *status = ST_NONE;

  while (d->pending != LEN_DONE) {
    int at_end_check = 0;

    if (d->need_rc_init) {
      while (avail > 0 && d->tmp_n < 5) {
        d->tmp[d->tmp_n++] = *src++;
        (*src_len)++;
        avail--;
      }
      if (d->tmp_n < 5) { *status = ST_MORE_INPUT; return RES_OK; }
      if (d->tmp[0] != 0) return RES_DATA;
      d->code = ((uint32_t)d->tmp[1] << 24) | ((uint32_t)d->tmp[2] << 16) |
                ((uint32_t)d->tmp[3] << 8) | (uint32_t)d->tmp[4];
      d->range = 0xFFFFFFFFu;
      d->need_rc_init = 0;
      d->tmp_n = 0;
    }

    if (d->dic_pos >= dic_limit) {
      if (d->pending == 0 && d->code == 0) { *status = ST_MAYBE_DONE; return RES_OK; }
      if (fin == FIN_ANY) { *status = ST_NOT_DONE; return RES_OK; }
      if (d->pending != 0) { *status = ST_NOT_DONE; return RES_DATA; }
      at_end_check = 1;
    }

    if (d->need_state_init) orc_init_state_real(d);

    if (d->tmp_n == 0) {
      const uint8_t *in_limit;
      size_t used;
      if (avail < LOOKAHEAD_MAX || at_end_check) {
        int k = orc_probe(d, src, avail);
        if (k == PROBE_SHORT) {
          memcpy(d->tmp, src, avail);
          d->tmp_n = (unsigned)avail;
          *src_len += avail;
          *status = ST_MORE_INPUT;
          return RES_OK;
        }
        if (at_end_check && k != PROBE_MATCH) { *status = ST_NOT_DONE; return RES_DATA; }
        in_limit = src;
      } else {
        in_limit = src + avail - LOOKAHEAD_MAX;
      }
      d->in = src;
      if (orc_run_split(d, dic_limit, in_limit) != RES_OK) return RES_DATA;
      used = (size_t)(d->in - src);
      *src_len += used;
      src += used;
      avail -= used;
    } else {
      unsigned have = d->tmp_n, taken = 0;
      while (have < LOOKAHEAD_MAX && taken < avail) d->tmp[have++] = src[taken++];
      d->tmp_n = have;
      if (have < LOOKAHEAD_MAX || at_end_check) {
        int k = orc_probe(d, d->tmp, have);
        if (k == PROBE_SHORT) {
          *src_len += taken;
          *status = ST_MORE_INPUT;
          return RES_OK;
        }
        if (at_end_check && k != PROBE_MATCH) { *status = ST_NOT_DONE; return RES_DATA; }
      }
      d->in = d->tmp;
      if (orc_run_split(d, dic_limit, d->in) != RES_OK) return RES_DATA;
      taken -= (have - (unsigned)(d->in - d->tmp));
      *src_len += taken;
      src += taken;
      avail -= taken;
      d->tmp_n = 0;
    }
  }
  if (d->code == 0) *status = ST_DONE_MARK;
  return d->code == 0 ? RES_OK : RES_DATA;
}

/* LzmaDec_DecodeToBuf (LzmaDec.c:840-878): ring dictionary -> caller buffer. */
static int orc_decode_to_buf(orc_dec *d, uint8_t *dest, size_t *dest_len,
                             const uint8_t *src, size_t *src_len, int fin, int *status) {
  size_t out_left = *dest_len, in_left = *src_len;
  *src_len = 0;
  *dest_len = 0;
  for (;;) {
    size_t in_cur = in_left, lim, start, produced;
    int cur_fin, res;
    if (d->dic_pos == d->dic_cap) d->dic_pos = 0;
    start = d->dic_pos;
    if (out_left > d->dic_cap - start) {
      lim = d->dic_cap;
      cur_fin = FIN_ANY;
    } else {
      lim = start + out_left;
      cur_fin = fin;
    }
    res = orc_decode_to_dic(d, lim, src, &in_cur, cur_fin, status);
    src += in_cur;
    in_left -= in_cur;
    *src_len += in_cur;
    produced = d->dic_pos - start;
    memcpy(dest, d->dic + start, produced);
    dest += produced;
    out_left -= produced;
    *dest_len += produced;
    if (res != RES_OK) return res;
    if (produced == 0 || out_left == 0) return RES_OK;
  }
}

int orc_lzma_decode(uint8_t *dst, size_t *dst_len, const uint8_t *src, size_t *src_len,
                    const uint8_t *props, unsigned props_size, int finish_mode,
                    int *status) {
  orc_dec d;
  size_t in_size = *src_len, out_size = *dst_len;
  int res;
  *status = -1;
  *src_len = 0;
  *dst_len = 0;
  if (in_size < 5) return RES_INPUT_EOF;
  memset(&d, 0, sizeof d);
  res = orc_props_parse(&d.pr, props, props_size);
  if (res != RES_OK) return res;
  d.nprobs = orc_num_probs(&d.pr);
  d.probs = (uint16_t *)malloc((size_t)d.nprobs * sizeof(uint16_t));
  if (!d.probs) return RES_MEM;
  d.dic = dst;
  d.dic_cap = out_size;
  orc_init(&d);
  *src_len = in_size;
  res = orc_decode_to_dic(&d, out_size, src, src_len, finish_mode, status);
  if (res == RES_OK && *status == ST_MORE_INPUT) res = RES_INPUT_EOF;
  *dst_len = d.dic_pos;
  free(d.probs);
  return res;
}

int orc_lzma_uncompress(uint8_t *dst, size_t *dst_len, const uint8_t *src,
                        size_t *src_len, const uint8_t *props, size_t props_size) {
  int st;
  return orc_lzma_decode(dst, dst_len, src, src_len, props, (unsigned)props_size,
                         FIN_ANY, &st);
}

int orc_lzma_stream_decode(const uint8_t *props, const uint8_t *src, size_t src_total,
                           uint8_t *out, size_t out_total, size_t in_chunk,
                           size_t out_chunk, int finish_mode, long long *trace,
                           int max_calls, size_t *out_len, size_t *in_used) {
  orc_dec d;
  size_t in_pos = 0, out_pos = 0;
  int calls = 0, res;
  memset(&d, 0, sizeof d);
  res = orc_props_parse(&d.pr, props, 5);
  if (res != RES_OK) { *out_len = 0; *in_used = 0; return -res; }
  d.nprobs = orc_num_probs(&d.pr);
  d.probs = (uint16_t *)malloc((size_t)d.nprobs * sizeof(uint16_t));
  d.dic_cap = d.pr.dict_size;
  d.dic = (uint8_t *)malloc(d.dic_cap);
  if (!d.probs || !d.dic) {
    free(d.probs);
    free(d.dic);
    *out_len = 0;
    *in_used = 0;
    return -RES_MEM;
  }
  orc_init(&d);
  while (calls < max_calls) {
    size_t sl = src_total - in_pos, dl = out_total - out_pos;
    int st = -1;
    if (sl > in_chunk) sl = in_chunk;
    if (dl > out_chunk) dl = out_chunk;
    res = orc_decode_to_buf(&d, out + out_pos, &dl, src + in_pos, &sl, finish_mode, &st);
    trace[4 * calls + 0] = res;
    trace[4 * calls + 1] = st;
    trace[4 * calls + 2] = (long long)sl;
    trace[4 * calls + 3] = (long long)dl;
    calls++;
    in_pos += sl;
    out_pos += dl;
    if (res != RES_OK) break;
    if (st == ST_DONE_MARK) break;
    if (out_pos == out_total) break;
    if (sl == 0 && dl == 0) break;
  }
  free(d.probs);
  free(d.dic);
  *out_len = out_pos;
  *in_used = in_pos;
  return calls;
}

/* The 7zDec.c:127-171 (SzDecodeLzma) loop: dic = the caller's whole output
 * buffer, LzmaDec_DecodeToDic(out_total, FINISH_END) over look windows of at
 * most `win` input bytes -- same contract as ref_lzma_dic_decode in
 * ref_lzma_shim.c (trace = {res, status, srcLen, dicPos} per call). */
int orc_lzma_dic_decode(const uint8_t *props, const uint8_t *src, size_t src_total,
                        uint8_t *out, size_t out_total, size_t win, long long *trace,
                        int max_calls, size_t *out_len, size_t *in_used) {
  orc_dec d;
  size_t in_pos = 0;
  int calls = 0, res;
  memset(&d, 0, sizeof d);
  res = orc_props_parse(&d.pr, props, 5);
  if (res != RES_OK) { *out_len = 0; *in_used = 0; return -res; }
  d.nprobs = orc_num_probs(&d.pr);
  d.probs = (uint16_t *)malloc((size_t)d.nprobs * sizeof(uint16_t));
  if (!d.probs) { *out_len = 0; *in_used = 0; return -RES_MEM; }
  d.dic = out;
  d.dic_cap = out_total;
  orc_init(&d);
  while (calls < max_calls) {
    size_t sl = src_total - in_pos, pos0 = d.dic_pos;
    int st = -1;
    if (sl > win) sl = win;
    res = orc_decode_to_dic(&d, out_total, src + in_pos, &sl, FIN_END, &st);
    if (trace) {
      trace[4 * calls + 0] = res;
      trace[4 * calls + 1] = st;
      trace[4 * calls + 2] = (long long)sl;
      trace[4 * calls + 3] = (long long)d.dic_pos;
    }
    calls++;
    in_pos += sl;
    if (res != RES_OK) break;
    if (d.dic_pos == d.dic_cap || (sl == 0 && d.dic_pos == pos0)) break;
  }
  free(d.probs);
  *out_len = d.dic_pos;
  *in_used = in_pos;
  return calls;
}

/* ---------------------------------------------------------------- LZMA2 */

enum {
  C2_CONTROL, C2_UNPACK0, C2_UNPACK1, C2_PACK0, C2_PACK1, C2_PROP, C2_DATA, C2_DATA_CONT,
  C2_FINISHED, C2_ERROR
};

typedef struct {
  orc_dec dec;
  uint32_t pack_left, unpack_left;
  int phase;
  uint8_t control;
  int need_dic_reset, need_state_reset, need_props;
} orc2_dec;

#define C2_IS_COPY(c) (((c) & 0x80) == 0)
#define C2_MODE(c) (((c) >> 5) & 3)

/* Chunk-header byte state machine (Lzma2Dec.c:98-157). */
static int orc2_header_byte(orc2_dec *p, uint8_t b) {
  switch (p->phase) {
    case C2_CONTROL:
      p->control = b;
      if (b == 0) return C2_FINISHED;
      if (C2_IS_COPY(b)) {
        if ((b & 0x7F) > 2) return C2_ERROR;
        p->unpack_left = 0;
      } else {
        p->unpack_left = (uint32_t)(b & 0x1F) << 16;
      }
      return C2_UNPACK0;
    case C2_UNPACK0:
      p->unpack_left |= (uint32_t)b << 8;
      return C2_UNPACK1;
    case C2_UNPACK1:
      p->unpack_left |= b;
      p->unpack_left++;
      return C2_IS_COPY(p->control) ? C2_DATA : C2_PACK0;
    case C2_PACK0:
      p->pack_left = (uint32_t)b << 8;
      return C2_PACK1;
    case C2_PACK1:
      p->pack_left |= b;
      p->pack_left++;
      if (C2_MODE(p->control) >= 2) return C2_PROP;
      return p->need_props ? C2_ERROR : C2_DATA;
    case C2_PROP: {
      unsigned lc, lp;
      if (b >= 225) return C2_ERROR;
      lc = b % 9;
      b /= 9;
      p->dec.pr.pb = b / 5;
      lp = b % 5;
      if (lc + lp > 4) return C2_ERROR;
      p->dec.pr.lc = lc;
      p->dec.pr.lp = lp;
      p->need_props = 0;
      return C2_DATA;
    }
  }
  return C2_ERROR;
}

static int orc2_decode_to_dic(orc2_dec *p, size_t dic_limit, const uint8_t *src,
                              size_t *src_len, int fin, int *status) {
  size_t in_size = *src_len;
  *src_len = 0;
  *status = ST_NONE;
  while (p->phase != C2_FINISHED) {
    size_t pos0 = p->dec.dic_pos;
    if (p->phase == C2_ERROR) return RES_DATA;
    if (pos0 == dic_limit && fin == FIN_ANY) { *status = ST_NOT_DONE; return RES_OK; }
    if (p->phase != C2_DATA && p->phase != C2_DATA_CONT) {
      if (*src_len == in_size) { *status = ST_MORE_INPUT; return RES_OK; }
      (*src_len)++;
      p->phase = orc2_header_byte(p, *src++);
      continue;
    }
    {
      size_t out_cur = dic_limit - pos0;
      size_t in_cur = in_size - *src_len;
      int cur_fin = FIN_ANY;
      if (p->unpack_left <= out_cur) {
        out_cur = p->unpack_left;
        cur_fin = FIN_END;
      }
      if (C2_IS_COPY(p->control)) {
        if (*src_len == in_size) { *status = ST_MORE_INPUT; return RES_OK; }
        if (p->phase == C2_DATA) {
          int reset = (p->control == 1);
          if (reset)
            p->need_props = p->need_state_reset = 1;
          else if (p->need_dic_reset)
            return RES_DATA;
          p->need_dic_reset = 0;
          orc_init_dic_state(&p->dec, reset, 0);
        }
        if (in_cur > out_cur) in_cur = out_cur;
        if (in_cur == 0) return RES_DATA;
        /* stored chunk (Lzma2Dec.c:159-166) */
        memcpy(p->dec.dic + p->dec.dic_pos, src, in_cur);
        p->dec.dic_pos += in_cur;
        if (p->dec.full == 0 && p->dec.pr.dict_size - p->dec.total <= in_cur)
          p->dec.full = p->dec.pr.dict_size;
        p->dec.total += (uint32_t)in_cur;
        src += in_cur;
        *src_len += in_cur;
        p->unpack_left -= (uint32_t)in_cur;
        p->phase = (p->unpack_left == 0) ? C2_CONTROL : C2_DATA_CONT;
      } else {
        size_t produced;
        int res;
        if (p->phase == C2_DATA) {
          int mode = C2_MODE(p->control);
          int init_dic = (mode == 3), init_state = (mode > 0);
          if ((!init_dic && p->need_dic_reset) || (!init_state && p->need_state_reset))
            return RES_DATA;
          orc_init_dic_state(&p->dec, init_dic, init_state);
          p->need_dic_reset = 0;
          p->need_state_reset = 0;
          p->phase = C2_DATA_CONT;
        }
        if (in_cur > p->pack_left) in_cur = p->pack_left;
        res = orc_decode_to_dic(&p->dec, pos0 + out_cur, src, &in_cur, cur_fin, status);
        src += in_cur;
        *src_len += in_cur;
        p->pack_left -= (uint32_t)in_cur;
        produced = p->dec.dic_pos - pos0;
        p->unpack_left -= (uint32_t)produced;
        if (res != RES_OK) return res;
        if (*status == ST_MORE_INPUT) return res;
        if (in_cur == 0 && produced == 0) {
          if (*status != ST_MAYBE_DONE || p->unpack_left != 0 || p->pack_left != 0)
            return RES_DATA;
          p->phase = C2_CONTROL;
        }
        if (*status == ST_MAYBE_DONE) *status = ST_NOT_DONE;
      }
    }
  }
  *status = ST_DONE_MARK;
  return RES_OK;
}

int orc_lzma2_decode(uint8_t *dst, size_t *dst_len, const uint8_t *src, size_t *src_len,
                     uint8_t prop, int finish_mode, int *status) {
  orc2_dec p;
  uint32_t dict;
  size_t sl = *src_len;
  int res;
  memset(&p, 0, sizeof p);
  *status = -1;
  if (prop > 40) { *dst_len = 0; *src_len = 0; return RES_UNSUPPORTED; }
  dict = (prop == 40) ? 0xFFFFFFFFu : ((2u | (prop & 1u)) << (prop / 2 + 11));
  /* Lzma2Dec_GetOldProps: lc+lp budget of 4 for allocation, dict as above */
  p.dec.pr.lc = 4;
  p.dec.pr.lp = 0;
  p.dec.pr.pb = 0;
  p.dec.pr.dict_size = dict < 4096 ? 4096 : dict;
  p.dec.nprobs = orc_num_probs(&p.dec.pr);
  p.dec.probs = (uint16_t *)malloc((size_t)p.dec.nprobs * sizeof(uint16_t));
  if (!p.dec.probs) return RES_MEM;
  p.dec.dic = dst;
  p.dec.dic_cap = *dst_len;
  /* Lzma2Dec_Init (Lzma2Dec.c:90-97) */
  p.phase = C2_CONTROL;
  p.need_dic_reset = p.need_state_reset = p.need_props = 1;
  orc_init(&p.dec);
  res = orc2_decode_to_dic(&p, *dst_len, src, &sl, finish_mode, status);
  *dst_len = p.dec.dic_pos;
  *src_len = sl;
  free(p.dec.probs);
  return res;
}

/* ---------------------------------------------------------------- batch (CPU baseline) */

typedef struct {
  const uint8_t *src;
  const uint64_t *src_off, *src_len;
  const uint8_t *props5;
  uint8_t *dst;
  const uint64_t *dst_off, *dst_cap;
  int fin;
  int32_t *res_out, *status_out;
  uint64_t *dest_len_out, *src_len_out;
  size_t n;
  size_t next;
  pthread_mutex_t mu;
  int errors;
} orc_batch;

static void *orc_batch_worker(void *arg) {
  orc_batch *b = (orc_batch *)arg;
  int errs = 0;
  for (;;) {
    size_t i, end, k;
    pthread_mutex_lock(&b->mu);
    i = b->next;
    end = i + 16 < b->n ? i + 16 : b->n;
    b->next = end;
    pthread_mutex_unlock(&b->mu);
    if (i >= b->n) break;
    for (k = i; k < end; k++) {
      size_t dl = b->dst_cap[k], sl = b->src_len[k];
      int st;
      int r = orc_lzma_decode(b->dst + b->dst_off[k], &dl, b->src + b->src_off[k], &sl,
                              b->props5 + 5 * k, 5, b->fin, &st);
      if (b->res_out) b->res_out[k] = r;
      if (b->status_out) b->status_out[k] = st;
      if (b->dest_len_out) b->dest_len_out[k] = dl;
      if (b->src_len_out) b->src_len_out[k] = sl;
      if (r != RES_OK) errs++;
    }
  }
  pthread_mutex_lock(&b->mu);
  b->errors += errs;
  pthread_mutex_unlock(&b->mu);
  return NULL;
}

int orc_lzma_decode_batch(const uint8_t *src, const uint64_t *src_off,
                          const uint64_t *src_len, const uint8_t *props5,
                          uint8_t *dst, const uint64_t *dst_off, const uint64_t *dst_cap,
                          int finish_mode, int32_t *res_out, int32_t *status_out,
                          uint64_t *dest_len_out, uint64_t *src_len_out, size_t n,
                          int threads) {
  orc_batch b;
  pthread_t tid[256];
  int t;
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  b.src = src;
  b.src_off = src_off;
  b.src_len = src_len;
  b.props5 = props5;
  b.dst = dst;
  b.dst_off = dst_off;
  b.dst_cap = dst_cap;
  b.fin = finish_mode;
  b.res_out = res_out;
  b.status_out = status_out;
  b.dest_len_out = dest_len_out;
  b.src_len_out = src_len_out;
  b.n = n;
  b.next = 0;
  b.errors = 0;
  pthread_mutex_init(&b.mu, NULL);
  if (threads == 1) {
    orc_batch_worker(&b);
  } else {
    for (t = 0; t < threads; t++) pthread_create(&tid[t], NULL, orc_batch_worker, &b);
    for (t = 0; t < threads; t++) pthread_join(tid[t], NULL);
  }
  pthread_mutex_destroy(&b.mu);
  return b.errors;
}

/* ------------------------------------------------------------------ CRC-32 */

static uint32_t orc_crc_table[256];
static pthread_once_t orc_crc_once = PTHREAD_ONCE_INIT;

/* table of 7zCrc.c:56-65 (CrcGenerateTable, first 256 entries) */
static void orc_crc_init(void) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t r = i;
    for (int j = 0; j < 8; j++) r = (r >> 1) ^ ((r & 1u) ? 0xEDB88320u : 0u);
    orc_crc_table[i] = r;
  }
}

uint32_t orc_crc_update(uint32_t crc, const uint8_t *data, size_t size) {
  pthread_once(&orc_crc_once, orc_crc_init);
  for (size_t i = 0; i < size; i++) crc = orc_crc_table[(crc ^ data[i]) & 0xFFu] ^ (crc >> 8);
  return crc;
}

uint32_t orc_crc_calc(const uint8_t *data, size_t size) {
  return orc_crc_update(0xFFFFFFFFu, data, size) ^ 0xFFFFFFFFu;
}
