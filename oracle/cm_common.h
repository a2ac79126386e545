/* cm_common.h — TEST ORACLE ONLY (never linked into the product).
 *
 * The adaptive frequency list (c_simple_model.h:63-171) and the carry-less
 * range coder (c_range_coder.h:20-164) shared by the fqzcomp_qual oracle
 * (fqz_oracle.c) and the sequence CM oracle (seq_oracle.c).
 */
#pragma once
#include <stdint.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* adaptive frequency list (c_simple_model.h)                          */
/* ------------------------------------------------------------------ */
#define FL_CAP_MAX 65519u   /* (1<<16)-17: halve when the total exceeds it */
#define FL_STEP    16u

/* Slot 0 is a permanent head whose frequency never loses a comparison, so
 * the one-step bubble never moves past it; slots 1..cap hold the symbols
 * in approximate descending frequency; slot cap+1 is a zero terminator and
 * slot cap+2 a maximal one that ends a decode scan past the symbols. */
typedef struct {
    uint32_t total;
    uint16_t fr[260];
    uint16_t sy[260];
} flist;

static inline void fl_init(flist *m, int cap, int live) {
    m->fr[0] = FL_CAP_MAX;
    m->sy[0] = 0;
    for (int k = 0; k < cap; k++) {
        m->sy[k + 1] = (uint16_t)k;
        m->fr[k + 1] = k < live ? 1 : 0;
    }
    m->fr[cap + 1] = 0;
    m->sy[cap + 1] = 0;
    m->fr[cap + 2] = FL_CAP_MAX;
    m->sy[cap + 2] = 0;
    m->total = (uint32_t)live;
}

/* halve every slot up to the first zero (c_simple_model.h:106-115) */
static inline void fl_halve(flist *m) {
    uint32_t t = 0;
    for (int k = 1; m->fr[k]; k++) {
        m->fr[k] = (uint16_t)(m->fr[k] - (m->fr[k] >> 1));
        t += m->fr[k];
    }
    m->total = t;
}

/* after coding slot k: bump, maybe halve, then one bubble step */
static inline int fl_bump(flist *m, int k) {
    m->fr[k] += FL_STEP;
    m->total += FL_STEP;
    if (m->total > FL_CAP_MAX) fl_halve(m);
    if (m->fr[k] > m->fr[k - 1]) {
        uint16_t f = m->fr[k], s = m->sy[k];
        m->fr[k] = m->fr[k - 1];
        m->sy[k] = m->sy[k - 1];
        m->fr[k - 1] = f;
        m->sy[k - 1] = s;
        return k - 1;
    }
    return k;
}

/* ------------------------------------------------------------------ */
/* range coder (c_range_coder.h)                                        */
/* ------------------------------------------------------------------ */
#define RC_TOP (1u << 24)

typedef struct {
    uint32_t lo, rng, code;
    uint32_t ffrun, pend, carry;   /* FF run length, pending byte, carry */
    uint8_t *p, *start, *end;
    int err;
} rcoder;

static inline void rc_enc_start(rcoder *c, uint8_t *out) {
    memset(c, 0, sizeof *c);
    c->rng = 0xFFFFFFFFu;
    c->p = c->start = out;
}

/* emit the pending byte (+carry) and any FF run, or extend the run */
static inline void rc_shift(rcoder *c) {
    if (c->lo < 0xFF000000u || c->carry) {
        *c->p++ = (uint8_t)(c->pend + c->carry);
        for (; c->ffrun; c->ffrun--) *c->p++ = (uint8_t)(c->carry - 1);
        c->pend = c->lo >> 24;
        c->carry = 0;
    } else {
        c->ffrun++;
    }
    c->lo <<= 8;
}

static inline void rc_put(rcoder *c, uint32_t cum, uint32_t f, uint32_t tot) {
    uint32_t before = c->lo;
    c->rng /= tot;
    c->lo += cum * c->rng;
    c->rng *= f;
    c->carry += c->lo < before;
    while (c->rng < RC_TOP) {
        c->rng <<= 8;
        rc_shift(c);
    }
}

static inline void rc_enc_finish(rcoder *c) {
    for (int k = 0; k < 5; k++) rc_shift(c);
}

static inline void rc_dec_start(rcoder *c, uint8_t *in, uint8_t *end) {
    memset(c, 0, sizeof *c);
    c->rng = 0xFFFFFFFFu;
    c->p = in;
    c->end = end;
    if (in + 5 > end) { c->p = end; return; }
    for (int k = 0; k < 5; k++) c->code = (c->code << 8) | *c->p++;
}

static inline uint32_t rc_target(rcoder *c, uint32_t tot) {
    if (!tot || c->rng < tot) return 0;
    c->rng /= tot;
    return c->code / c->rng;
}

static inline void rc_take(rcoder *c, uint32_t cum, uint32_t f) {
    c->code -= cum * c->rng;
    c->rng *= f;
    while (c->rng < RC_TOP) {
        if (c->p >= c->end) { c->err = -1; return; }
        c->code = (c->code << 8) + *c->p++;
        c->rng <<= 8;
    }
}

/* code / decode one symbol of a list with capacity `cap` */
static inline void fl_encode(flist *m, rcoder *c, unsigned sym) {
    uint32_t acc = 0;
    int k = 1;
    while (m->sy[k] != sym) acc += m->fr[k++];
    rc_put(c, acc, m->fr[k], m->total);
    fl_bump(m, k);
}

static inline unsigned fl_decode(flist *m, rcoder *c, int cap) {
    uint32_t t = rc_target(c, m->total);
    if (t > FL_CAP_MAX) return 0;
    uint32_t acc = 0;
    int k = 1;
    while ((acc += m->fr[k]) <= t) k++;
    if (k - 1 > cap) return 0;
    acc -= m->fr[k];
    rc_take(c, acc, m->fr[k]);
    unsigned s = m->sy[k];
    fl_bump(m, k);
    return s;
}

