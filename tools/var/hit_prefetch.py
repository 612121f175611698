# A/B patch: a bounced ray's hit record (its sphere's centre and material lines) touched right after the
# sweep, one dword of each XORed into one VGPR that next_ray consumes, so next_ray's gather of the record
# finds the lines in L1/L2 after terminate and the camera batches instead of waiting on them.
import sys
d = sys.argv[1]
p = f"{d}/rt_trace.hpp"; s = open(p).read()
old = """        if (act) hit_i = nearest_hit<T, ROOT2, SC, false, MEGA>(p, o, d, hit_t);"""
new = """        if (act) hit_i = nearest_hit<T, ROOT2, SC, false, MEGA>(p, o, d, hit_t);
        if (act && hit_i >= 0) {
            const auto& qh = *cold_args<T>();
            hpf = ((const uint32_t*)(qh.mats + hit_i))[0] ^ ((const uint32_t*)(qh.cen + 4 * hit_i))[0];
        }"""
assert old in s; s = s.replace(old, new)
old = """        if (fresh || scat) {
            const uint32_t ssv = ss_get();
            const uint32_t pix = (!CAMQ && fresh) ? npix : s_slotpix[wave][slot_of(ssv)];"""
new = """        asm volatile("" ::"v"(hpf));
        if (fresh || scat) {
            const uint32_t ssv = ss_get();
            const uint32_t pix = (!CAMQ && fresh) ? npix : s_slotpix[wave][slot_of(ssv)];"""
assert old in s; s = s.replace(old, new)
old = """    for (;;) {
        bool fresh = false;"""
new = """    uint32_t hpf = 0;   // hit-record prefetch (consumed by the next next_ray)
    for (;;) {
        bool fresh = false;"""
assert s.count(old) == 1; s = s.replace(old, new)
open(p, "w").write(s)
