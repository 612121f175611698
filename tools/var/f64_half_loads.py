# A/B patch: fp64 exact4 loads only the 64-B half groups holding a sphere some lane passes.
import sys
d = sys.argv[1]
p = f"{d}/rt_sweep.hpp"; s = open(p).read()
old = '''            } else {
                const SphGroup<T> c0 = load_group(fe, 2 * g), c1 = load_group(fe, 2 * g + 1);
                T hb[4], disc[4];
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    if (!((pairs >> j) & 1u)) continue;'''
new = '''            } else {
                SphGroup<T> c0, c1;
                if (pairs & 3u) c0 = load_group(fe, 2 * g);
                if (pairs & 12u) c1 = load_group(fe, 2 * g + 1);
                T hb[4], disc[4];
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    if (!((pairs >> j) & 1u)) continue;'''
assert old in s, "exact4 fp64"; s = s.replace(old, new); open(p, "w").write(s)
