// rt-render — the reference's binary (src/main.rs:27-74) on the MI355X sample loop.
//
//   rt-render [--scene scene.toml] [--width 3840] [--height 2160] [--spp 100] [--bounces 50]
//             [--seed 0x5EED0001] [--f32] [--root2] [--mode vectorized2|vectorized|vectorized3|scalar]
//             [--out output.png|.ppm] [--block-size B] [--dump-scene]
//
// --mode picks which of the reference's renderers is reproduced (include/rt_mi355x.h): the live
// render_vectorized2 (default), render_vectorized, or the scalar render.
//
// Defaults are main.rs's hard-coded values (scene.toml in the working directory, 3840x2160, 50
// bounces, 100 spp, camera from (16,2,18.5) looking at the origin, vfov 30, focal 10, no defocus,
// output.png).  --dump-scene prints the flattened scene as JSON and exits (no GPU needed).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>

#include "image.hpp"
#include "scene.hpp"

using namespace rt_host;

// Rust's `{}` for f64: the shortest representation that round-trips.
static std::string rs(double v) {
    if (v == std::floor(v) && std::fabs(v) < 1e15) {
        std::ostringstream o;
        o << (long long)v;
        if (v == 0 && std::signbit(v)) return "-0";
        return o.str();
    }
    for (int p = 1; p <= 17; ++p) {
        char buf[64];
        std::snprintf(buf, sizeof buf, "%.*g", p, v);
        if (std::strtod(buf, nullptr) == v) {
            std::string s(buf);
            if (s.find('e') == std::string::npos) return s;
            std::snprintf(buf, sizeof buf, "%.17f", v);   // Rust never prints exponents for {}
            s = buf;
            while (!s.empty() && s.back() == '0') s.pop_back();
            return s;
        }
    }
    return std::to_string(v);
}
static std::string rs3(const double* v) { return "[" + rs(v[0]) + ", " + rs(v[1]) + ", " + rs(v[2]) + "]"; }

static void dump_scene(const Scene& sc) {
    FlatScene f = sc.flatten();
    std::printf("{\"n_spheres\": %zu, \"center\": [", f.radius.size());
    for (size_t i = 0; i < f.center.size(); ++i) std::printf("%s%.17g", i ? ", " : "", f.center[i]);
    std::printf("], \"radius\": [");
    for (size_t i = 0; i < f.radius.size(); ++i) std::printf("%s%.17g", i ? ", " : "", f.radius[i]);
    std::printf("], \"material\": [");
    for (size_t i = 0; i < f.material.size(); ++i) std::printf("%s%u", i ? ", " : "", f.material[i]);
    std::printf("], \"materials\": [");
    for (size_t i = 0; i < f.materials.size(); ++i) {
        const rt_material& m = f.materials[i];
        std::printf("%s{\"kind\": %u, \"hollow\": %u, \"albedo\": [%.17g, %.17g, %.17g], \"fuzz\": %.17g, \"ior\": %.17g}",
                    i ? ", " : "", m.kind, m.hollow, m.albedo[0], m.albedo[1], m.albedo[2], m.fuzz, m.ior);
    }
    std::printf("]}\n");
}

int main(int argc, char** argv) {
    std::string scene_path = "scene.toml", out = "output.png";
    uint32_t width = 3840, height = 2160, spp = 100, bounces = 50, flags = 0, block_size = 0;
    uint64_t seed = 0x5EED0001ull;
    bool dump = false;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&]() -> std::string {
            if (i + 1 >= argc) { std::fprintf(stderr, "missing value for %s\n", a.c_str()); std::exit(2); }
            return argv[++i];
        };
        if (a == "--scene") scene_path = next();
        else if (a == "--width") width = (uint32_t)std::stoul(next());
        else if (a == "--height") height = (uint32_t)std::stoul(next());
        else if (a == "--spp") spp = (uint32_t)std::stoul(next());
        else if (a == "--bounces") bounces = (uint32_t)std::stoul(next());
        else if (a == "--seed") seed = std::stoull(next(), nullptr, 0);
        else if (a == "--f32") flags |= RT_FLAG_F32;
        else if (a == "--root2") flags |= RT_FLAG_ROOT2;
        else if (a == "--mode") {
            const std::string m = next();
            flags &= ~(RT_FLAG_MODE_VECTORIZED | RT_FLAG_MODE_SCALAR | RT_FLAG_MODE_VECTORIZED3);
            if (m == "vectorized") flags |= RT_FLAG_MODE_VECTORIZED;
            else if (m == "vectorized3") flags |= RT_FLAG_MODE_VECTORIZED3;
            else if (m == "scalar") flags |= RT_FLAG_MODE_SCALAR;
            else if (m != "vectorized2") { std::fprintf(stderr, "unknown mode %s\n", m.c_str()); return 2; }
        }
        else if (a == "--out") out = next();
        else if (a == "--block-size") block_size = (uint32_t)std::stoul(next());
        else if (a == "--dump-scene") dump = true;
        else if (a == "-h" || a == "--help") {
            std::puts("rt-render [--scene scene.toml] [--width W] [--height H] [--spp S] [--bounces B] [--seed N] "
                      "[--f32] [--root2] [--mode vectorized2|vectorized|vectorized3|scalar] [--out output.png] [--block-size B] "
                      "[--dump-scene]");
            return 0;
        } else { std::fprintf(stderr, "unknown argument %s\n", a.c_str()); return 2; }
    }
    try {
        std::ifstream in(scene_path, std::ios::binary);   // main.rs:31-34
        if (!in) throw Panic("Can't read scene from file " + scene_path);
        std::stringstream ss;
        ss << in.rdbuf();
        Scene scene;
        try {
            scene = scene_from_toml(ss.str());
        } catch (const toml::ParseError& e) {
            throw Panic("Failed parsing scene from file " + scene_path + ": " + e.what());   // main.rs:36-39
        }
        if (dump) { dump_scene(scene); return 0; }

        const double from[3] = {16.0, 2.0, 18.5};   // main.rs:51-58
        Camera camera(width, height, 10.0, 30.0, Vec3{16.0, 2.0, 18.5}, Vec3{0, 0, 0}, Vec3{0, 1, 0}, 0.0);
        const double vh = std::tan((30.0 * (3.141592653589793 / 180.0)) / 2.0) * 10.0 * 2.0;   // ray_tracing.rs:29
        std::printf("Parameters:\n");                                                          // ray_tracing.rs:46-50
        std::printf("\tCamera Center:            %s\n", rs3(from).c_str());
        std::printf("\tViewport Height:          %s\n", rs(vh).c_str());
        std::printf("\tViewport Width:           %s\n", rs(vh * ((double)width / (double)height)).c_str());
        std::printf("\tViewport Top Left Corner: %s\n", rs3(camera.c.ulc).c_str());
        std::printf("\t Number of objects: \t %zu\n", scene.len());                           // main.rs:60

        GpuRenderer renderer(seed, flags, block_size);   // block_size 128: TileRenderer::new(None, 128), main.rs:62
        std::fprintf(stderr, "Rendering %u by %u image on %s (%s)...\n", width, height, rt_version(),
                     (flags & RT_FLAG_F32) ? "fp32" : "fp64");
        auto [image, stat] = renderer.render(bounces, spp, scene, camera);                     // main.rs:64
        save_image(out, image.width, image.height, image.data.data());                         // main.rs:66
        std::printf("Image Size: %u x %u\n", camera.image_width(), camera.image_height());    // main.rs:68-71
        std::printf("Total Pixels: %zu\n", stat.pixels_rendered);
        std::printf("Time Taken: %.3f seconds\n", stat.duration.count());
        std::printf("Average Pixel Rate: %.2f px/s\n", stat.pixels_per_second);
        std::printf("Sample Rate: %.2f Msamples/s (kernel %.3f ms, %llu ray segments)\n",
                    (double)stat.gpu.samples / stat.duration.count() / 1e6, stat.gpu.kernel_ms,
                    (unsigned long long)stat.gpu.ray_segments);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "thread 'main' panicked: %s\n", e.what());
        return 101;   // Rust's panic exit status
    }
    return 0;
}
