# A/B patch: the bit-plane comparator of finish_pixel's replay on 32-bit halves with v_bitop3 / v_and_or
# (11 VALU per plane instead of ~22: the compiler built the 64-bit lane masks with cndmasks).
import sys
d = sys.argv[1]
p = f"{d}/rt_finish.hpp"; s = open(p).read()
old = '''                unsigned long long eq = inm, gt = 0ull, eqk = inm;
                uint32_t zb = 0;
                for (uint32_t bb = nb; bb-- > 0u;) {
                    const unsigned long long P = __ballot(in && ((ec >> bb) & 1u));
                    if (P == 0ull) { zb |= 1u << bb; continue; }
                    const unsigned long long B = ((ec >> bb) & 1u) ? ~0ull : 0ull;     // this lane's bit
                    const unsigned long long Bk = ((lane >> bb) & 1u) ? ~0ull : 0ull;  // bit of k = lane
                    gt |= eq & P & ~B;     // equal so far, 1 where this lane has 0: greater
                    eq &= ~(P ^ B);        // still equal
                    eqk &= ~(P ^ Bk);
                }'''
new = '''                // the masks as 32-bit halves: B, Bk are all-ones or zero per lane (v_bfe_i32), each update
                // one v_bitop3 / v_and_or per half (truth table index = S0 << 2 | S1 << 1 | S2)
                uint32_t eql = (uint32_t)inm, eqh = (uint32_t)(inm >> 32), gtl = 0u, gth = 0u;
                uint32_t eqkl = eql, eqkh = eqh;
                // Unconditional per plane (no branch, no loop-carried copies): a plane no lane sets leaves eq
                // and gt unchanged in the lanes that use them and clears eqk in the lanes k with that bit.
                const uint32_t zb = 0;
                for (uint32_t bb = nb; bb-- > 0u;) {
                    const uint32_t B = (uint32_t)__builtin_amdgcn_sbfe((int)ec, bb, 1u);     // this lane's bit
                    const unsigned long long P = __ballot(B != 0u) & inm;
                    const uint32_t Pl = (uint32_t)P, Ph = (uint32_t)(P >> 32);
                    const uint32_t Bk = (uint32_t)__builtin_amdgcn_sbfe((int)lane, bb, 1u);  // bit of k = lane
                    // gt |= eq & P & ~B (equal so far, 1 where this lane has 0: greater)
                    gtl = ((eql & ~B) & Pl) | gtl;
                    gth = ((eqh & ~B) & Ph) | gth;
                    // eq &= ~(P ^ B) (still equal), eqk &= ~(P ^ Bk): table 0x90
                    eql = __builtin_amdgcn_bitop3_b32(eql, Pl, B, 0x90);
                    eqh = __builtin_amdgcn_bitop3_b32(eqh, Ph, B, 0x90);
                    eqkl = __builtin_amdgcn_bitop3_b32(eqkl, Pl, Bk, 0x90);
                    eqkh = __builtin_amdgcn_bitop3_b32(eqkh, Ph, Bk, 0x90);
                }
                const unsigned long long eq = ((unsigned long long)eqh << 32) | eql;
                const unsigned long long gt = ((unsigned long long)gth << 32) | gtl;
                const unsigned long long eqk = ((unsigned long long)eqkh << 32) | eqkl;'''
assert old in s; s = s.replace(old, new); open(p, "w").write(s)
