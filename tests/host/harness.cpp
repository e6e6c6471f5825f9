// Host build of the DEVICE arithmetic (consensus_overlord_amd/csrc/bls/*.hpp) for CPU unit
// tests against the golden fixtures. Test infrastructure only: never linked into the
// product library, never a fallback.
#include <string.h>
#include "../../consensus_overlord_amd/csrc/bls/verify.hpp"
#include "../../consensus_overlord_amd/csrc/fpvm.hpp"
#include "../../consensus_overlord_amd/csrc/rlp.hpp"

using namespace ovh;

static const uint8_t DST[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_";

extern "C" {

// rlp(Vote) + SM3 of rlp.hpp (the k_vote_digest code) on the host
int hx_vote_rlp(uint8_t* out, uint64_t h, uint64_t r, uint8_t t, const uint8_t* bh, uint32_t bl) {
  return (int)rlp_vote(out, h, r, t, bh, bl);
}
void hx_vote_digest(uint8_t* out32, uint64_t h, uint64_t r, uint8_t t, const uint8_t* bh, uint32_t bl) {
  vote_digest(out32, h, r, t, bh, bl);
}

int hx_hash_to_g2(const uint8_t* msg32, const uint8_t* dst, uint32_t dst_len, uint8_t* out192) {
  XmdTemplates t;
  if (!xmd_build_templates(t, dst, dst_len)) return -1;
  uint32_t m[8];
  be_words_from_bytes(m, msg32, 8);
  G2J h;
  hash_to_g2(h, m, t);
  g2_serialize(out192, h);
  return 0;
}

int hx_verify(const uint8_t* sig, uint32_t sl, const uint8_t* hash, uint32_t hl, const uint8_t* pk, uint32_t pl) {
  XmdTemplates t;
  xmd_build_templates(t, DST, 43);
  return verify_one(sig, sl, hash, hl, pk, pl, t);
}

int hx_g1_decode(const uint8_t* in, uint32_t len, uint8_t* out48, int* inf) {
  G1A a;
  bool i;
  int e = g1_from_bytes(a, i, in, len);
  *inf = i;
  if (e == 0) {
    G1J j;
    if (i) jac_set_inf(j); else jac_from_aff(j, a);
    g1_compress(out48, j);
  }
  return e;
}

int hx_g2_decode(const uint8_t* in, uint32_t len, uint8_t* out96, int* inf) {
  G2A a;
  bool i;
  int e = g2_from_bytes(a, i, in, len);
  *inf = i;
  if (e == 0) {
    G2J j;
    if (i) jac_set_inf(j); else jac_from_aff(j, a);
    g2_compress(out96, j);
  }
  return e;
}

// e(G1, G2)^3 via the device Miller loop + x-chain final exponentiation; 12 Fp2 coeffs
// (c0.c0.c0, c0.c0.c1, c0.c1.c0, ...) as 48-byte BE canonical values.
void hx_gt_g1g2(uint8_t* out576) {
  G1A p; fp_load(p.x, G1X_M); fp_load(p.y, G1Y_M);
  G2A q; q.x = fp2_const(G2X_C0, G2X_C1); q.y = fp2_const(G2Y_C0, G2Y_C1);
  Fp12 f;
  miller_loop(f, p, q);
  final_exponentiation(f, f);
  const Fp* c = &f.c0.c0.c0;
  for (int i = 0; i < 12; ++i) fp_to_be48(out576 + 48 * i, c[i]);
}

int hx_g2_subgroup(const uint8_t* in, uint32_t len) {
  G2A a; bool i;
  int e = g2_from_bytes(a, i, in, len);
  if (e) return -e;
  G2J j; jac_from_aff(j, a);
  return g2_in_subgroup(j) ? 1 : 0;
}

int hx_g1_subgroup(const uint8_t* in, uint32_t len) {
  G1A a; bool i;
  int e = g1_from_bytes(a, i, in, len);
  if (e) return -e;
  G1J j; jac_from_aff(j, a);
  return g1_in_subgroup(j) ? 1 : 0;
}

// The VM's modular inverse (fpvm.hpp fp_inv) on a raw canonical value: r3 = raw R turns the
// closing Montgomery product into the identity, so out = a^-1 mod p (0 -> 0).
void hx_fp_inv_raw(const uint32_t* a, const uint32_t* r_raw, uint32_t* out) {
  Fp x, r, rr;
  for (int k = 0; k < 12; ++k) x.v[k] = a[k], rr.v[k] = r_raw[k];
  ovh::vm::fp_inv(r, x, rr);
  for (int k = 0; k < 12; ++k) out[k] = r.v[k];
}

// One slice of an Fp-VM program through the interpreter (fpvm.hpp exec), lane by lane in each
// phase (a phase's writes never target a slot that phase reads: tools/fpvm/sched.py).
// slots: nslots x 12 words (in/out); planes: `st` output planes, 12 words each.
// any_all = 1 runs every wave-uniform block for every lane (all phase-header bits set).
// side / scr (spilled programs, fpvm.hpp run<true>): per-lane side words and the unit's
// scratch; after a phase's ops, its spills store their slots, then the next phase's fills land.
int hx_vm_run(const uint32_t* code, uint32_t nphases, uint32_t W, uint32_t NW, const uint32_t* cst, uint32_t* slots,
              uint64_t scalar, uint32_t* planes, uint32_t nplanes, int any_all, const uint32_t* side, uint32_t* scr) {
  using namespace ovh::vm;
  const uint32_t all =
      any_all ? (H_MUL | H_MULNEG | H_FLAG | H_LIN | H_LINNEG | H_LINNEG2 | H_LINNEG3 | H_ACC | H_RARE | H_SELB) : 0u;
  const ovh::vm::Out out{planes, 1, 0};
  (void)nplanes;
  for (uint32_t ph = 0; ph < nphases; ++ph) {
    if (ph > 0 && side)
      for (uint32_t lane = 0; lane < W; ++lane) {
        const uint32_t sw = side[(size_t)(ph - 1) * W + lane];
        if ((sw >> 30) == 2)  // spill of phase ph - 1
          for (int k = 0; k < 12; ++k) scr[((sw >> 11) & 0xFFF) * 12 + k] = slots[(sw & 0x7FF) * 12 + k];
      }
    if (ph > 0 && side)
      for (uint32_t lane = 0; lane < W; ++lane) {
        const uint32_t sw = side[(size_t)ph * W + lane];
        if ((sw >> 30) == 3)  // fill of phase ph
          for (int k = 0; k < 12; ++k) slots[(sw & 0x7FF) * 12 + k] = scr[((sw >> 11) & 0xFFF) * 12 + k];
      }
    for (uint32_t lane = 0; lane < W; ++lane) {
      const uint32_t* w = code + ((size_t)ph * W + lane) * NW;
      ovh::vm::exec(uint4{w[0] | all, w[1], w[2], w[3]}, true, slots, cst, scalar, out);
      // the interpreter's lazy-reduction invariant: every slot result lies in [0, 2p)
      const uint32_t op = w[0] & 31, dst = (w[0] >> 5) & 0x7FF;
      if (op != ovh::vm::OP_NOP && op != ovh::vm::OP_ST) {
        uint32_t br = 0;
        for (int k = 0; k < 12; ++k) (void)subc32(slots[dst * 12 + k], ovh::vm::P2_LIMBS[k], br, &br);
        if (!br) return -1 - (int)ph;
      }
    }
  }
  return 0;
}

}
