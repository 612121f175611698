// scene.hpp — C++ host mirror of the reference's host-side surface, above the C ABI:
//   Vec3/Color::from_toml, toml_utils::to_float        src/geometry.rs:190-211, src/color.rs:99-123,
//                                                       src/toml_utils.rs:2-12
//   Material (Lambertian / Metal / Dielectric)          src/materials.rs:12-155
//   Object::Sphere, get_object_list                     src/objects.rs:17-52, 203-300
//   Scene, Camera::new                                  src/ray_tracing.rs:27-62, 100-104, 217-229
//   Renderer, RenderStat                                src/renderer.rs:11-40
// Where the reference panics (unwrap / panic! / Index on a missing key), these throw rt_host::Panic
// with the reference's message.
#pragma once
#include <algorithm>
#include <cctype>
#include <chrono>
#include <cstring>
#include <map>
#include <memory>
#include <optional>
#include <string>
#include <utility>
#include <vector>

#include "../../include/rt_mi355x.h"
#include "toml.hpp"

namespace rt_host {

struct Panic : std::runtime_error {
    using std::runtime_error::runtime_error;
};

inline const toml::Value& index(const toml::Table& t, const std::string& k) {   // Index<&str> for Map
    auto it = t.find(k);
    if (it == t.end()) throw Panic("index not found: key \"" + k + "\" missing from table");
    return it->second;
}
template <typename T> T unwrap(const std::optional<T>& o, const char* what) {
    if (!o) throw Panic(std::string("called `Option::unwrap()` on a `None` value (") + what + ")");
    return *o;
}
inline std::string lower(std::string s) {
    for (auto& c : s) c = (char)std::tolower((unsigned char)c);
    return s;
}

// toml_utils.rs:2-12
inline std::optional<double> to_float(const toml::Value& v) {
    if (v.is_float()) return v.f;
    if (v.is_int()) return (double)v.i;
    return std::nullopt;
}

struct Vec3 {
    double x = 0, y = 0, z = 0;
    // geometry.rs:190-211
    static std::optional<Vec3> from_toml(const toml::Value& v) {
        if (auto* t = v.as_table())
            return Vec3{unwrap(to_float(index(*t, "x")), "x"), unwrap(to_float(index(*t, "y")), "y"),
                        unwrap(to_float(index(*t, "z")), "z")};
        if (auto* a = v.as_array()) {
            if (a->size() < 3) throw Panic("assertion failed: array.len() >= 3");
            return Vec3{unwrap(to_float((*a)[0]), "x"), unwrap(to_float((*a)[1]), "y"), unwrap(to_float((*a)[2]), "z")};
        }
        return std::nullopt;
    }
};

struct Color {
    double red = 0, green = 0, blue = 0;
    // color.rs:99-123 (table entries that are not numbers read as 0.0; missing keys panic)
    static std::optional<Color> from_toml(const toml::Value& v) {
        if (auto* t = v.as_table())
            return Color{to_float(index(*t, "red")).value_or(0.0), to_float(index(*t, "green")).value_or(0.0),
                         to_float(index(*t, "blue")).value_or(0.0)};
        if (auto* a = v.as_array()) {
            if (a->size() < 3) throw Panic("assertion failed: array.len() >= 3");
            return Color{unwrap(to_float((*a)[0]), "red"), unwrap(to_float((*a)[1]), "green"),
                         unwrap(to_float((*a)[2]), "blue")};
        }
        return std::nullopt;
    }
};

// trait Material (materials.rs:35-39); to_rt() flattens a material for the C ABI.
struct Material {
    virtual ~Material() = default;
    virtual rt_material to_rt() const = 0;
};

struct Lambertian : Material {   // materials.rs:41-69
    Color albedo;
    explicit Lambertian(Color a) : albedo(a) {}
    rt_material to_rt() const override {
        rt_material m{};
        m.kind = RT_LAMBERTIAN;
        m.albedo[0] = albedo.red; m.albedo[1] = albedo.green; m.albedo[2] = albedo.blue;
        return m;
    }
    static std::shared_ptr<Material> from_table(const toml::Table& t) {
        return std::make_shared<Lambertian>(unwrap(Color::from_toml(index(t, "albedo")), "albedo"));
    }
};

struct Metal : Material {   // materials.rs:71-107
    Color albedo;
    double fuzzy_factor;
    Metal(Color a, double f) : albedo(a), fuzzy_factor(rt_metal_clamp_fuzz(f)) {}   // Metal::new clamp
    rt_material to_rt() const override {
        rt_material m{};
        m.kind = RT_METAL;
        m.albedo[0] = albedo.red; m.albedo[1] = albedo.green; m.albedo[2] = albedo.blue;
        m.fuzz = fuzzy_factor;
        return m;
    }
    static std::shared_ptr<Material> from_table(const toml::Table& t) {
        return std::make_shared<Metal>(unwrap(Color::from_toml(index(t, "albedo")), "albedo"),
                                       unwrap(to_float(index(t, "fuzzy_factor")), "fuzzy_factor"));
    }
};

struct Dielectric : Material {   // materials.rs:109-155
    double index_of_refraction;
    bool hollow;
    Dielectric(double ior, bool h) : index_of_refraction(ior), hollow(h) {}
    rt_material to_rt() const override {
        rt_material m{};
        m.kind = RT_DIELECTRIC;
        m.hollow = hollow ? 1u : 0u;
        m.ior = index_of_refraction;
        return m;
    }
    static std::shared_ptr<Material> from_table(const toml::Table& t) {
        const toml::Value& h = index(t, "hollow");
        if (!h.is_bool()) throw Panic("called `Option::unwrap()` on a `None` value (hollow)");
        return std::make_shared<Dielectric>(unwrap(to_float(index(t, "index_of_refraction")), "index_of_refraction"), h.b);
    }
};

using MaterialTable = std::map<std::string, std::shared_ptr<Material>>;

// materials.rs:21-33
inline std::shared_ptr<Material> load_material_from_toml(const toml::Table& t) {
    const std::string* ty = index(t, "type").as_str();
    if (!ty) throw Panic("called `Option::unwrap()` on a `None` value (type)");
    const std::string k = lower(*ty);
    if (k == "lambertian") return Lambertian::from_table(t);
    if (k == "metal") return Metal::from_table(t);
    if (k == "dielectric") return Dielectric::from_table(t);
    throw Panic("Unknown material type " + k + "!");
}

// materials.rs:12-19
inline MaterialTable get_materials(const toml::Table& t) {
    MaterialTable out;
    for (const auto& [key, value] : t) {
        const toml::Table* mt = value.as_table();
        if (!mt) throw Panic("called `Option::unwrap()` on a `None` value (material table)");
        out.emplace(key, load_material_from_toml(*mt));
    }
    return out;
}

struct Sphere {   // objects.rs:203-214, 292-299
    Vec3 center;
    double radius;
    std::shared_ptr<Material> material;
    static Sphere from_table(const toml::Table& t, const MaterialTable& mats) {
        Vec3 c = unwrap(Vec3::from_toml(index(t, "center")), "center");
        double r = unwrap(to_float(index(t, "radius")), "radius");
        const std::string* name = index(t, "material").as_str();
        if (!name) throw Panic("called `Option::unwrap()` on a `None` value (material)");
        auto it = mats.find(*name);
        if (it == mats.end()) throw Panic("called `Option::unwrap()` on a `None` value (material \"" + *name + "\")");
        return Sphere{c, r, it->second};
    }
};

// objects.rs:38-52
inline Sphere load_object_from_toml(const toml::Table& t, const MaterialTable& mats) {
    const std::string* ty = index(t, "type").as_str();
    if (!ty) throw Panic("called `Option::unwrap()` on a `None` value (type)");
    const std::string k = lower(*ty);
    if (k == "sphere") return Sphere::from_table(t, mats);
    throw Panic("Unknown object type " + k);
}
inline std::vector<Sphere> get_object_list(const toml::Array& a, const MaterialTable& mats) {
    std::vector<Sphere> out;
    for (const auto& v : a) {
        const toml::Table* t = v.as_table();
        if (!t) throw Panic("called `Option::unwrap()` on a `None` value (hitable)");
        out.push_back(load_object_from_toml(*t, mats));
    }
    return out;
}

// Owning SoA image of a Scene in the C-ABI layout (scene order kept: ties -> later sphere).
struct FlatScene {
    std::vector<double> center, radius;
    std::vector<uint32_t> material;
    std::vector<rt_material> materials;
    rt_scene view() const {
        rt_scene s{};
        s.n_spheres = (uint32_t)radius.size();
        s.n_materials = (uint32_t)materials.size();
        s.center = center.data(); s.radius = radius.data(); s.material = material.data();
        s.materials = materials.data();
        return s;
    }
};

struct Scene {   // ray_tracing.rs:100-104, 217-229, 308-310
    std::vector<Sphere> objects;
    static Scene from_list(const std::vector<Sphere>& l) { return Scene{l}; }
    void add(Sphere s) { objects.push_back(std::move(s)); }
    size_t len() const { return objects.size(); }
    FlatScene flatten() const {
        FlatScene f;
        std::map<const Material*, uint32_t> ids;
        for (const auto& s : objects) {
            auto [it, fresh] = ids.emplace(s.material.get(), (uint32_t)f.materials.size());
            if (fresh) f.materials.push_back(s.material->to_rt());
            f.center.insert(f.center.end(), {s.center.x, s.center.y, s.center.z});
            f.radius.push_back(s.radius);
            f.material.push_back(it->second);
        }
        return f;
    }
};

// src/main.rs:29-43: a scene file -> Scene
inline Scene scene_from_toml(const std::string& text) {
    toml::Value root = toml::parse(text);
    const toml::Table& r = *root.as_table();
    const toml::Table* mats = index(r, "materials").as_table();
    if (!mats) throw Panic("called `Option::unwrap()` on a `None` value (materials)");
    const toml::Array* hit = index(r, "hitables").as_array();
    if (!hit) throw Panic("called `Option::unwrap()` on a `None` value (hitables)");
    MaterialTable mt = get_materials(*mats);
    return Scene::from_list(get_object_list(*hit, mt));
}

struct Camera {   // ray_tracing.rs:27-62 via rt_camera_new
    rt_camera c{};
    Camera(uint32_t w, uint32_t h, double focal_length, double view_angle, Vec3 center, Vec3 look_at, Vec3 up,
           double defocus_angle) {
        const double ce[3] = {center.x, center.y, center.z}, la[3] = {look_at.x, look_at.y, look_at.z},
                     u[3] = {up.x, up.y, up.z};
        if (rt_camera_new(&c, w, h, focal_length, view_angle, ce, la, u, defocus_angle) != RT_OK)
            throw Panic(rt_last_error());
    }
    uint32_t image_width() const { return c.image_width; }
    uint32_t image_height() const { return c.image_height; }
};

struct RenderStat {   // renderer.rs:11-34
    std::chrono::duration<double> duration;
    size_t pixels_rendered;
    double pixels_per_second;
    rt_stats gpu;
    RenderStat(std::chrono::duration<double> d, size_t px, rt_stats g = {})
        : duration(d), pixels_rendered(px), pixels_per_second(px / d.count()), gpu(g) {}
};

struct RgbImage {
    uint32_t width = 0, height = 0;
    std::vector<uint8_t> data;   // row-major interleaved RGB8 (image::RgbImage raw layout)
};

struct Renderer {   // renderer.rs:38-40
    virtual ~Renderer() = default;
    virtual std::pair<RgbImage, RenderStat> render(size_t max_bounces, size_t samples_per_pixel, const Scene& scene,
                                                   const Camera& camera) = 0;
};

// The GPU implementation of Renderer (replaces TileRenderer, renderer.rs:232-387).
// block_size 0: the whole image in one launch (rt_render).  block_size B > 0: TileRenderer's
// decomposition (renderer.rs:248-266): B x B blocks, row-major, one launch each on one device
// context, and after each the reference's per-block line (renderer.rs:339), with the block's pixel
// rate from the launch's kernel time: "Device 0 complete block (x, y) at R px/s".  The image is the
// same either way (the RNG is keyed by the global pixel index).
struct GpuRenderer : Renderer {
    uint64_t seed;
    uint32_t flags;
    uint32_t block_size;
    explicit GpuRenderer(uint64_t s = 0x5EED0001ull, uint32_t f = 0, uint32_t b = 0) : seed(s), flags(f), block_size(b) {}
    std::pair<RgbImage, RenderStat> render(size_t max_bounces, size_t spp, const Scene& scene,
                                           const Camera& camera) override {
        const auto t0 = std::chrono::steady_clock::now();
        FlatScene flat = scene.flatten();
        rt_scene rs = flat.view();
        RgbImage img{camera.image_width(), camera.image_height(), {}};
        img.data.resize((size_t)img.width * img.height * 3);
        rt_stats st{};
        if (block_size == 0) {
            const int rc = rt_render(&rs, &camera.c, (uint32_t)max_bounces, (uint32_t)spp, seed, flags, nullptr,
                                     img.data.data(), nullptr, &st);
            if (rc == RT_ERR_RANGE) throw Panic(std::string("assertion failed: ") + rt_last_error());
            if (rc != RT_OK) throw Panic(std::string("rt_render failed: ") + rt_last_error());
        } else {
            render_blocks(rs, camera, (uint32_t)max_bounces, (uint32_t)spp, img, st);
        }
        const size_t npx = (size_t)img.width * img.height;
        RenderStat stat(std::chrono::steady_clock::now() - t0, npx, st);
        return {std::move(img), stat};
    }

  private:
    void render_blocks(const rt_scene& rs, const Camera& camera, uint32_t max_bounces, uint32_t spp, RgbImage& img,
                       rt_stats& total) {
        struct Ctx {
            rt_context* c = nullptr;
            void* buf = nullptr;
            ~Ctx() { if (buf) rt_device_free(c, buf); if (c) rt_context_destroy(c); }
        } x;
        auto chk = [](int rc, const char* what) {
            if (rc == RT_ERR_RANGE) throw Panic(std::string("assertion failed: ") + rt_last_error());
            if (rc != RT_OK) throw Panic(std::string(what) + ": " + rt_last_error());
        };
        chk(rt_context_create(0, &x.c), "rt_context_create");
        chk(rt_context_set_scene(x.c, &rs), "rt_context_set_scene");
        const uint32_t B = block_size, W = img.width, H = img.height;
        chk(rt_device_alloc(x.c, (size_t)B * B * 3, &x.buf), "rt_device_alloc");
        std::vector<uint8_t> tile((size_t)B * B * 3);
        const uint32_t nbx = (W + B - 1) / B, nby = (H + B - 1) / B;   // renderer.rs:248-266
        bool range_err = false;
        for (uint32_t by = 0; by < nby; ++by)
            for (uint32_t bx = 0; bx < nbx; ++bx) {
                const uint32_t c0 = bx * B, r0 = by * B;
                const rt_tile_range tr{r0, 1, std::min(B, H - r0), c0, std::min(B, W - c0)};
                chk(rt_render_async(x.c, &camera.c, max_bounces, spp, seed, flags, &tr, x.buf, nullptr, nullptr),
                    "rt_render_async");
                rt_stats st{};
                const int rc = rt_context_collect(x.c, nullptr, &st);
                if (rc == RT_ERR_RANGE) range_err = true;
                else chk(rc, "rt_context_collect");
                const size_t npx = (size_t)tr.row_count * tr.col_count;
                chk(rt_memcpy_d2h(x.c, tile.data(), x.buf, npx * 3), "rt_memcpy_d2h");
                for (uint32_t r = 0; r < tr.row_count; ++r)
                    std::memcpy(&img.data[((size_t)(r0 + r) * W + c0) * 3], &tile[(size_t)r * tr.col_count * 3],
                                (size_t)tr.col_count * 3);
                // renderer.rs:339: "Thread {} complete block ({}, {}) at {:.2} px/s"
                std::printf("Device 0 complete block (%u, %u) at %.2f px/s\n", bx, by, st.pixels_per_second);
                total.kernel_ms += st.kernel_ms;
                total.pixels += st.pixels;
                total.samples += st.samples;
                total.ray_segments += st.ray_segments;
                total.lane_slots += st.lane_slots;
                total.direct_sky_samples += st.direct_sky_samples;
                total.bounce_iters += st.bounce_iters;
            }
        if (range_err) throw Panic("assertion failed: a pixel channel exceeded 2.0 (color.rs:55-57)");
    }
};

}  // namespace rt_host
