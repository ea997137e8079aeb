// dse_wht.h -- descriptors of the Walsh-Hadamard engine (dse_wht.hip): H|w> for registers of
// more than two tiles as D_Z + W D_X W + V D_Y V^+ in a few streaming passes over HBM.
#pragma once

#include "dse_internal.h"

namespace dse {

// WHT_FINAL_NEXT: FINAL of term k, then the next term's FIRST from the new w_k still in registers
// (option wht_fuse)
enum { WHT_FIRST = 0, WHT_FWD = 1, WHT_MID = 2, WHT_INV = 3, WHT_FINAL = 4, WHT_FINAL_NEXT = 5 };

constexpr int kWhtMinTile = 12;                       // tile bits of the passes: 12 or 13
constexpr int kWhtMaxTile = 13;
constexpr int kWhtMaxGroups = 4;                      // group 0 + up to 3 high groups
constexpr int kWhtMaxOuter = DSE_MAX_HIGH_BITS(12);   // 22 outer bits at 34 qubits
constexpr int kWhtMaxQubits = 34;

// Tile bit q of a group-g tile is global bit pos[q]; outer index bit i is global bit opos[i].
// Group 0: pos = 0..WL-1.  High groups: pos[0..c-1] = 0..c-1 (carried, not transformed in this
// pass: contiguous 2^c-amplitude runs keep the loads coalesced), pos[c..WL-1] = the group's bits.
struct WhtGroup {
  int pos[kWhtMaxTile];
  int c;
  int n_outer;
  int opos[kWhtMaxOuter];
};

struct WhtProb {
  double2* vec_a;         // W-basis image of w (X branch)
  double2* vec_b;         // V-basis image of w (Y branch)
  // Partitioned register (shard r of 2^S, local bits n_local = n - S): the MID pass runs on the
  // index-swapped copies (vec_at, vec_bt: local top S bits <-> shard bits, an all-to-all between
  // the shards); gmap[local bit] = global bit in that state, the global bits then held by the
  // rank index are fix_mask with values fix_val.  Unpartitioned: vec_*t = vec_*, gmap = identity.
  double2* vec_at;
  double2* vec_bt;
  uint64_t fix_mask, fix_val;
  int gmap[kWhtMaxQubits];
  int phase0;             // popcount of the rank's global bits (S phases of FIRST / FINAL)
  const double* cquad;    // [n*n] symmetric: (pair_ij / 2) * 2^-n, zero diagonal
  // per-tile coefficient tables (launch_wht_tables), one row per outer index o:
  double* ztab;           // [tiles][16] group 0: F_i(o) i < WL, C(o) without beta (D_Z, s = 1/2 - bit)
  double* xytab;          // [tiles][32] MID group: F^X_q(o), C^X(o) at 0..WL, F^Y, C^Y at 16..16+WL
  // Tile-independent pair forms per thread (launch_wht_tables): form 0 = MID's in-tile pair
  // couplings in MID's diagonal layout, form 1 = FINAL's in-tile zz / 4 in layout B; each
  // [5][NT] (qt, qh[0..3] of every thread) then zr[16] (register-register part per r).
  double* qtab;
  double lin_x[kWhtMaxQubits];  // Re c_1 of the drive of bit b, * 2^-n
  double lin_y[kWhtMaxQubits];  // Im c_1, * 2^-n
  int n;                  // qubits of the whole register
  int n_local;            // qubits held in this context (n - S)
  int wl;                 // tile bits (== DevProb::L)
  int n_groups;
  WhtGroup grp[kWhtMaxGroups];
};

// Fills ztab / xytab of problem wp (device pointers to one WhtProb / DevProb entry).
hipError_t launch_wht_tables(int wl, const WhtProb* wp, const DevProb* dp, int64_t tiles, hipStream_t st);

// One H application (mode MODE_APPLY) or one Chebyshev term (MODE_FIRST / MODE_GEN, buffer
// roles and coefficient rows as launch_step) over items (problem, tile index), in three parts:
//   pre  = FIRST, FWD over groups 1..G-2      mid = MID (group G-1)      post = INV, FINAL
// (partitioned registers swap vec_* <-> vec_*t between the parts).  Every item's problem has
// P.L == wl.  vsel selects the vectors (1: the X-branch A, 2: the Y-branch B, 3: both): pre with
// vsel 1 = FIRST + FWD(A), 2 = FWD(B); mid = MID(vsel); post with vsel 1 = INV(A), 2 = INV(B) +
// FINAL -- so a partitioned register can swap one vector while the other is transformed.
enum { WHT_PART_PRE = 0, WHT_PART_MID = 1, WHT_PART_POST = 2 };
// pgrid > 0 with pmask bit 1: MID as a persistent launch of pgrid workgroups (k_wht_mid_p)
hipError_t launch_wht_part(int part, int wl, int mode, int n_groups, const WhtProb* wp, const DevProb* dp,
                           const int2* items, int n_items, int k, int q, int set, int vsel, hipStream_t st,
                           int pgrid = 0, int pmask = 0);

}  // namespace dse
