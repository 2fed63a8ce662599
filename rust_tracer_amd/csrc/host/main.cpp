// main.cpp -- `rust_tracer` command line front-end over the C ABI.
//
// The reference CLI (src/cli.rs:34-175) and its modes (src/main.rs:27-291), minus the GTK
// GUI and the terminal preview:
//   rust_tracer [-w W] [-h H] [-d D] [--method basic|rayforest] [--stats] [-i]
//               [--scene my_scene|bench128|synth2|synth3] [--device N] [--out FILE]
//   rust_tracer [...] bench [-n RUNS] [-f]
// Normal mode renders once and saves ./output/<unix seconds>.png (main.rs:71-74,
// bmp.rs:8-19: RGB8 from Color::as_u8), or --out FILE (.png, .bmp or .ppm).  With
// --method rayforest it builds the forest, optionally prints RayForest::stats
// (main.rs:88-103) and saves render_forest's image.  Bench mode prints the same
// "Total Time" / "Avg Per Op" lines as main.rs:137-219: RUNS renders, RUNS forest shades,
// or with -f RUNS render_forest_filter calls for the shape named "blue".
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <sys/stat.h>
#include <vector>

#include "scene.hpp"

using namespace rust_tracer;

namespace {

typedef std::chrono::steady_clock Clock;

long long ms_since(Clock::time_point t0) {
    return (long long)std::chrono::duration_cast<std::chrono::milliseconds>(Clock::now() - t0).count();
}

bool save(const std::string& path, const std::vector<uint8_t>& rgb8, uint32_t w, uint32_t h) {
    return rt_write_image(path.c_str(), rgb8.data(), w, h) == RT_OK;
}

// Color::as_u8 (color.rs:43-46) on the host for the forest path's float frames
void as_u8(const std::vector<float>& rgb, std::vector<uint8_t>& out) {
    out.resize(rgb.size());
    for (size_t i = 0; i < rgb.size(); i++) {
        float x = 255.f * rgb[i];
        out[i] = x >= 255.f ? 255 : (x > 0.f ? (uint8_t)x : 0);  // `as u8` saturates, NaN -> 0
    }
}

void enter_to_proceed() {  // main.rs:125-131
    std::printf("Enter To Proceed: ");
    std::fflush(stdout);
    char buf[256];
    if (!std::fgets(buf, sizeof buf, stdin)) return;
}

void usage() {
    std::fprintf(stderr,
                 "usage: rust_tracer [-w W] [-h H] [-d D] [--method basic|rayforest] [--stats] [-i]\n"
                 "                   [--scene my_scene|bench128|synth2|synth3|synth5] [--device N] [--out FILE]\n"
                 "                   [--spp N] [--seed S]\n"
                 "                   [bench [-n RUNS] [-f]]\n");
}

int fail(const char* what, rt_status st) {
    std::fprintf(stderr, "%s: %s\n", what, rt_status_str(st));
    return 1;
}

}  // namespace

int main(int argc, char** argv) {
    uint32_t w = 512, h = 512, depth = 8;  // cli.rs defaults
    int device = -1, runs = 10;
    uint32_t spp = 1, seed = 0;  // supersampling (config 5; not in the reference CLI)
    bool bench = false, forest_method = false, stats = false, interactive = false, filter = false;
    std::string scene_name = "my_scene", out;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        auto next = [&]() -> const char* {
            if (i + 1 >= argc) {
                usage();
                std::exit(2);
            }
            return argv[++i];
        };
        if (a == "-w" || a == "--width") w = (uint32_t)std::atoi(next());
        else if (a == "-h" || a == "--height") h = (uint32_t)std::atoi(next());
        else if (a == "-d" || a == "--depth") depth = (uint32_t)std::atoi(next());
        else if (a == "--scene") scene_name = next();
        else if (a == "--device") device = std::atoi(next());
        else if (a == "--spp") spp = (uint32_t)std::atoi(next());
        else if (a == "--seed") seed = (uint32_t)std::atoi(next());
        else if (a == "--out") out = next();
        else if (a == "--stats") stats = true;
        else if (a == "-i" || a == "--interactive") interactive = true;
        else if (a == "bench") bench = true;
        else if (a == "-n" || a == "--runs") runs = std::atoi(next());
        else if (a == "-f" || a == "--filter") filter = true;
        else if (a == "--method") {
            std::string m = next();
            for (auto& ch : m) ch = (char)std::tolower(ch);
            if (m == "rayforest") forest_method = true;
            else if (m == "basic") forest_method = false;
            else {
                std::fprintf(stderr, "Unexpected value provided for `--method`: %s\n", m.c_str());  // cli.rs:150
                return 2;
            }
        } else {
            usage();
            return 2;
        }
    }
    std::printf("Rendering configuration: Config { width: %u, height: %u, depth: %u, method: %s, interactive: %s, "
                "subcommand: %s, print_forest_stats: %s }\n",
                w, h, depth, forest_method ? "RayForest" : "Basic", interactive ? "true" : "false",
                bench ? "Benchmark" : "Normal", stats ? "true" : "false");
    std::printf("Create Scene\n");
    Scene scene;
    if (scene_name == "my_scene") create_scene(scene);
    else if (scene_name == "bench128") create_bench_128_scene(scene);
    else if (scene_name == "synth2" || scene_name == "synth3" || scene_name == "synth5") {
        rt_synth_params p;
        rt_synth_config(scene_name[5] - '0', &p);
        create_synth_scene(scene, p);
    } else {
        usage();
        return 2;
    }
    std::printf("Done Creating Scene\n");

    // a handle of its own for the forest and supersampling paths; the basic path renders
    // through render(), whose Scene keeps its device scene
    rt_scene* s = nullptr;
    rt_status st = RT_OK;
    if (forest_method || spp != 1) {
        auto flat = scene.flatten();
        st = rt_scene_create(&flat->desc, device, &s);
        if (st != RT_OK) return fail("rt_scene_create", st);
    }
    Camera cam(w, h);
    rt_camera c = cam.to_c();
    std::vector<float> rgb((size_t)w * h * 3);
    std::vector<uint8_t> rgb8((size_t)w * h * 3);
    if (out.empty() && !bench) {  // main.rs:71-74: ./output/<unix seconds>.png
        ::mkdir("./output", 0755);
        out = "./output/" + std::to_string((long long)std::time(nullptr)) + ".png";
    }
    if (interactive && !bench) enter_to_proceed();

    if (!forest_method) {
        rt_counters cnt;
        float kms = 0.f;
        rt_render_opts opts{device, &cnt, &kms};
        int n = bench ? runs : 1;
        RenderBuffer buffer(w, h);
        if (bench && spp == 1) {
            // the reference builds its scene before the timed loop (main.rs:35-38, 134-152):
            // the Scene's device scene is built by one untimed render() here, reported apart
            auto w0 = Clock::now();
            st = render(cam, scene, buffer, depth, device, &cnt, &kms);
            if (st != RT_OK) return fail("render", st);
            std::printf("device scene build + first render (untimed): %lldms\n", ms_since(w0));
        }
        auto t0 = Clock::now();
        for (int k = 0; k < n; k++) {
            auto r0 = Clock::now();
            if (spp == 1) {
                // render_scene_basic (main.rs:244-261): render() on the same Scene every call;
                // the Scene keeps its device scene (the first call builds it)
                st = render(cam, scene, buffer, depth, device, &cnt, &kms);
                if (st != RT_OK) return fail("render", st);
            } else {
                st = rt_render_spp(s, &c, depth, spp, seed, &opts, rgb.data(), rgb8.data());
                if (st != RT_OK) return fail("rt_render_spp", st);
            }
            std::printf("render_scene: %lldms\n", ms_since(r0));  // main.rs:250-253
        }
        if (spp == 1) {
            std::memcpy(rgb.data(), buffer.buf.data(), rgb.size() * sizeof(float));
            as_u8(rgb, rgb8);  // bmp.rs:8-19
        }
        long long ns = (long long)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t0).count();
        if (bench) {
            std::printf("Total Time: %lldms | %lldns\n", ns / 1000000, ns);
            std::printf("Avg Per Op: %gms | %gns\n", (double)(ns / 1000000) / n, (double)ns / n);
        }
        std::printf("rays: node %llu shadow %llu pixels %llu (kernel %.3f ms)\n", (unsigned long long)cnt.node_rays,
                    (unsigned long long)cnt.shadow_rays, (unsigned long long)cnt.pixels, kms);
    } else {
        if (bench) std::printf("This will benchmark evaluating the complete forest\n");
        std::printf("Rendering in RayForest Mode\nGenerate Forest\n");
        auto g0 = Clock::now();
        rt_forest* f = nullptr;
        st = rt_forest_create(s, &c, depth, &f);
        if (st != RT_OK) return fail("rt_forest_create", st);
        std::printf("generate_forest: %lldms\nDone Generating Forest\n", ms_since(g0));
        if (stats && !bench) {  // main.rs:88-103, render_tree.rs:73-93
            std::vector<uint32_t> sizes((size_t)w * h);
            st = rt_forest_tree_sizes(f, sizes.data());
            if (st != RT_OK) return fail("rt_forest_tree_sizes", st);
            std::vector<uint32_t> sorted(sizes);
            std::sort(sorted.begin(), sorted.end());
            size_t n = sorted.size();
            unsigned long long total = 0;
            for (uint32_t v : sorted) total += v;
            auto at = [&](float q) { return sorted[(size_t)(q * (float)n)]; };
            std::printf("Number of Trees: %zu\n", n);
            std::printf("Min Tree Size: %u\n", sorted.front());
            std::printf("Max Tree Size: %u\n", sorted.back());
            std::printf("Median Size: %u\n", sorted[n / 2]);
            std::printf("p90 Size: %u\n", at(0.9f));
            std::printf("p95 Size: %u\n", at(0.95f));
            std::printf("p99 Size: %u\n", at(0.99f));
            std::printf("Number of Intersections: %llu\n", total);
            std::printf("Number of Shapes: %zu\n", scene.size());
            std::printf("Number of Intersection Tests: %llu\n", (unsigned long long)scene.size() * total);
        }
        if (interactive && !bench) enter_to_proceed();
        if (!bench) {
            auto r0 = Clock::now();
            st = rt_forest_render(f, rgb.data());
            if (st != RT_OK) return fail("rt_forest_render", st);
            as_u8(rgb, rgb8);
            if (!save(out, rgb8, w, h)) {
                std::fprintf(stderr, "cannot write %s\n", out.c_str());
                return 1;
            }
            std::printf("render_forest_to_file: %lldms\n", ms_since(r0));
        } else {
            long long ns = 0;
            if (!filter) {
                std::printf("Render full forest\n");
                auto t0 = Clock::now();
                for (int k = 0; k < runs; k++) {
                    auto r0 = Clock::now();
                    st = rt_forest_render(f, rgb.data());
                    if (st != RT_OK) return fail("rt_forest_render", st);
                    std::printf("render_forest: %lldms\n", ms_since(r0));
                }
                ns = (long long)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t0).count();
            } else {
                std::printf("Render partial forest\n");
                const Shape* blue = scene.find_shape("blue");
                if (!blue) {
                    std::fprintf(stderr, "no shape named \"blue\" in this scene\n");
                    return 1;
                }
                int32_t id = blue->id;
                std::vector<float> buffer((size_t)w * h * 3, 0.f);  // RenderBuffer::new
                auto t0 = Clock::now();
                for (int k = 0; k < runs; k++) {
                    st = rt_forest_render_filter(f, &id, 1, buffer.data());
                    if (st != RT_OK) return fail("rt_forest_render_filter", st);
                }
                ns = (long long)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t0).count();
                uint64_t with = 0;
                st = rt_forest_trees_with(f, id, &with);
                if (st != RT_OK) return fail("rt_forest_trees_with", st);
                size_t trees = (size_t)w * h;
                std::printf("Forest Size: %zu\n", trees);
                std::printf("Trees Evaluated: %llu\n", (unsigned long long)with);
                std::printf("%% evaluated: %g\n", 100.f * (float)with / (float)trees);
            }
            std::printf("Total Time: %lldms | %lldns\n", ns / 1000000, ns);
            std::printf("Avg Per Op: %gms | %gns\n", (double)(ns / 1000000) / runs, (double)ns / runs);
        }
        rt_forest_destroy(f);
        rt_scene_destroy(s);
        return 0;
    }
    if (!bench || !out.empty()) {
        if (!out.empty() && !save(out, rgb8, w, h)) {
            std::fprintf(stderr, "cannot write %s\n", out.c_str());
            return 1;
        }
        if (!out.empty()) std::printf("wrote %s\n", out.c_str());
    }
    if (s) rt_scene_destroy(s);
    return 0;
}
