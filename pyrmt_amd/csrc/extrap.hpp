// extrap.hpp -- shared layout of the extrapolation workspace (extrap.hip: band detection and
// the row-ticket sweep used as the general fallback; extrap_chain.hip: the geometry-first
// chain path used whenever its capacity limits hold).
#pragma once
#include "rmt_internal.hpp"

namespace rmt {

typedef unsigned long long u64;

constexpr int EX_MAXL = 8;          // layers the chain path handles (more -> fallback sweep)
constexpr int CH_R = 2048;          // chain value ring (slots, chain order); deps < CH_R/2 back
#ifndef RMT_CH_W
#define RMT_CH_W 16
#endif
constexpr int CH_W = RMT_CH_W;      // chain workgroup waves (4 per SIMD)
constexpr int CH_HDR = 24;          // record header, doubles
constexpr int CH_TVS = 88;          // padded fold terms per sum (81 rounded up to 8)
constexpr int CH_MAXREC = 8 * (CH_HDR + 6 * CH_TVS + 4 * 64);   // 6464 B (<= 64 sources)
constexpr int EX_MAXREJ = 4096;     // rejected fits per layer the fix-up handles
constexpr int EX_DCAP = 8192;       // fix-up dirty-list capacity

// ctl words (int): fallback flag, abort flag, accepted count, and 64-bit arena cursor
// EXC_ANY / EXC_NOOP: k_ex_none's proof that no target can be accepted (both paths skip)
// EXC_CMIN / EXC_CMAX: column range of the targets; EXC_NPART + p: fits in chain part p,
// EXC_NPART + CH_MAXP: the number of parts = EXC_NCOL column ranges x EXC_NLG layer groups
constexpr int CH_MAXP = 8;          // chain parts (workgroups): target column range x layer group
enum { EXC_FALLBACK = 0, EXC_ABORT = 1, EXC_FILLED = 2, EXC_ARENA = 4, EXC_REJ = 8,
       EXC_BASE = 8 + EX_MAXL, EXC_ANY = 8 + 2 * EX_MAXL, EXC_NOOP = EXC_ANY + 1,
       EXC_CMIN = EXC_ANY + 2, EXC_CMAX = EXC_ANY + 3, EXC_NPART = EXC_ANY + 4,
       EXC_WSTART = EXC_NPART + CH_MAXP + 1,                // + p * CH_W + w: wave w's first
       EXC_NCOL = EXC_WSTART + CH_MAXP * CH_W,              // ordinal in part p
       EXC_NLG = EXC_NCOL + 1,
       EXC_WORDS = EXC_NLG + 8 };
// cross-part hand-off granules (gval) hold this signalling NaN until the fit is published: an
// arithmetic result is never a signalling NaN (IEEE mode), so the value is its own flag
constexpr unsigned long long CH_GSENT = 0x7ff00000000bad01ull;
// The abort word (status[1]) names what stopped: EXA_TAG | kind << 26 | part << 22 | id, with
// id the ordinal (within its part) of the chain fit whose wait timed out; the first abort of
// a call wins (CAS from 0).  Host side: extrap_abort_detail (rmt_internal.hpp).  (Naming the
// kind of wait inside the chain's fit cost the kernel a register spill at 128 VGPRs, so the
// chain reports its part and the stopped fit only.)
enum { EXA_CHAIN = 1, EXA_RELINK = 7, EXA_SWEEP = 8, EXA_PAR = 9 };
constexpr int EXA_TAG = 1 << 30;
__device__ __forceinline__ int exa_code(int kind, int part, int id) {
    return EXA_TAG | (kind << 26) | ((part & 15) << 22) | (id < 0 ? 0x3fffff : min(id, 0x3fffff));
}
__device__ __forceinline__ void exa_report(int *status, int code) {
    atomicCAS(status + 1, 0, code);
}
constexpr int PX_K = 64;            // parallel mode: fits per segment
constexpr int PX_F = 64;            // frontier capacity (more: the segment is solved serially)
constexpr int PX_S = 81;            // window sources per fit
constexpr int PX_H = 8;             // segment header ints
constexpr int PX_PB = 768;          // packed block of a segment for k_px_comb (doubles)

struct ExWs {
    // band detection (both paths) and the fallback sweep
    u64 *kbits, *cbits, *Kold;     // Kold: ML planes
    unsigned char *rowcand;
    int *jrange, *status;          // status[0] filled, [1] abort (fallback sweep)
    // chain path
    u64 *T, *ACC, *KN;             // ML planes each: targets, accepted, known after layer
    int *rowcnt, *rowoff, *wordoff, *cbase;   // ML*ny, ML*(ny+1), ML*ny*W, ML*ny
    long long *tcell, *recoff, *rec_by_chain; // MAXT each
    int *chain_of, *dmark;                    // MAXT each
    // parts: part[x] of chain index x, loc[x] its ordinal within the part, inv[base_p + l]
    // the chain index of ordinal l of part p (base_p = fits of the parts before p);
    // cross-part hand-offs go through L2 / the fabric: gval by global slot base_p + l, two
    // 8-byte granules (X1, X2) stored write-through, CH_GSENT until published (a record's
    // meta bit 63 marks a fit read by another part)
    unsigned char *part;                      // MAXT
    int *loc, *inv;                           // MAXT each
    // wave assignment: wnext[base_p + l] = the next ordinal of part p that ordinal l's wave
    // runs (round robin, k_ex_runs)
    int *wnext;                               // MAXT
    double *gval;                             // 2 * MAXT
    int *rej;                                 // ML * EX_MAXREJ
    int *ctl;                                 // EXC_WORDS
    // parallel mode (extrap_par.hip; laid out after everything else, only when requested):
    // per fit id the window sources in window order -- first the static ones (solid cells:
    // key = cell; earlier layers' fits: key = -(id + 1)), then the same-layer fits -- with
    // their coefficients beta; the fit values; per segment of PX_K consecutive ids of a layer
    // its frontier and its affine response (M^T, N^T) and the constants d = N c
    int *pns, *pnd;                           // MAXT each: static / same-layer source counts
    int *pkey;                                // MAXT * PX_S
    double *pbeta;                            // MAXT * PX_S
    double2 *pval, *pc;                       // MAXT each: fit values, static sums c
    unsigned char *live;                      // MAXT: read by a later segment's frontier
    int *shdr, *sF;                           // maxseg * PX_H, maxseg * PX_F
    double *sMT, *sNT;                        // maxseg * PX_F * PX_K, maxseg * PX_K * PX_K
    double2 *sd;                              // maxseg * PX_K
    double *spk;                              // maxseg * PX_PB: k_px_comb's packed blocks
    long maxseg;
    char *arena;
    long long arena_bytes;
    int slots;                                // 1: record of fit id at id * CH_MAXREC
    long maxt;
    long plane;                               // ny * W
};

// px: also lay out the parallel mode's arrays (after everything else: the other offsets do
// not depend on it)
ExWs extrap_layout(void *base, int ny, int nx, int max_layers, size_t *bytes, bool px = false,
                   bool bump = false);
// chain path: queue the kernels; they check ctl[EXC_FALLBACK] themselves
int extrap_chain_prep(rmt_ctx *ctx, const ExWs &ws, const double *X1o, const double *X2o,
                      double dx, double dy, int ML);
int extrap_chain_values(rmt_ctx *ctx, const ExWs &ws, const double *X1o, const double *X2o,
                        double dx, double dy, int ML);
int extrap_chain_run(rmt_ctx *ctx, const ExWs &ws, const double *X1o, const double *X2o, int ML);
bool extrap_chain_supported(int ny, int nx, int ML);
// chain prep without the chain-order passes and with no records (the parallel mode only
// needs targets and acceptance)
int extrap_chain_prep_px(rmt_ctx *ctx, const ExWs &ws, double dx, double dy, int ML);
// the parallel mode (extrap_par.hip): geometry after the acceptance passes, values after
// the map is advected
int extrap_par_geometry(rmt_ctx *ctx, const ExWs &ws, double dx, double dy, int ML);
int extrap_par_values(rmt_ctx *ctx, const ExWs &ws, double *X1o, double *X2o, int ML);

}  // namespace rmt
