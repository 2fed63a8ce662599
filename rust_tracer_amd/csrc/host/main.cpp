// main.cpp -- `rust_tracer` command line front-end over the C ABI.
//
// The subset of the reference CLI (src/cli.rs:34-118, src/main.rs:27-261) that drives
// the render path:
//   rust_tracer [-w W] [-h H] [-d D] [--scene my_scene|bench128|synth2|synth3]
//               [--device N] [--out FILE.bmp|.ppm]
//   rust_tracer [...] bench [-n RUNS]
// Normal mode renders once and writes the image (bmp.rs:8-19 writes RGB8 from
// Color::as_u8); bench mode repeats render_scene_basic RUNS times and prints the same
// "Total Time" / "Avg Per Op" lines as main.rs:137-151.  Timing covers the render call
// (scene upload excluded, as in main.rs:250-253).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "scene.hpp"

using namespace rust_tracer;

namespace {

bool write_bmp(const std::string& path, const std::vector<uint8_t>& rgb, uint32_t w, uint32_t h) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    uint32_t row = (w * 3 + 3) & ~3u;
    uint32_t size = 54 + row * h;
    uint8_t hdr[54] = {'B', 'M'};
    auto put32 = [&](int off, uint32_t v) {
        for (int i = 0; i < 4; i++) hdr[off + i] = (uint8_t)(v >> (8 * i));
    };
    put32(2, size);
    put32(10, 54);
    put32(14, 40);
    put32(18, w);
    put32(22, h);
    hdr[26] = 1;
    hdr[28] = 24;
    put32(34, row * h);
    std::fwrite(hdr, 1, 54, f);
    std::vector<uint8_t> line(row, 0);
    for (uint32_t y = 0; y < h; y++) {
        uint32_t v = h - 1 - y;  // bottom-up
        for (uint32_t u = 0; u < w; u++) {
            const uint8_t* p = &rgb[((size_t)v * w + u) * 3];
            line[u * 3 + 0] = p[2];
            line[u * 3 + 1] = p[1];
            line[u * 3 + 2] = p[0];
        }
        std::fwrite(line.data(), 1, row, f);
    }
    std::fclose(f);
    return true;
}

bool write_ppm(const std::string& path, const std::vector<uint8_t>& rgb, uint32_t w, uint32_t h) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    std::fprintf(f, "P6\n%u %u\n255\n", w, h);
    std::fwrite(rgb.data(), 1, rgb.size(), f);
    std::fclose(f);
    return true;
}

void usage() {
    std::fprintf(stderr,
                 "usage: rust_tracer [-w W] [-h H] [-d D] [--scene my_scene|bench128|synth2|synth3]\n"
                 "                   [--device N] [--out FILE] [bench [-n RUNS]]\n");
}

}  // namespace

int main(int argc, char** argv) {
    uint32_t w = 512, h = 512, depth = 8;  // cli.rs defaults
    int device = -1, runs = 10;
    bool bench = false;
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
        else if (a == "--out") out = next();
        else if (a == "bench") bench = true;
        else if (a == "-n" || a == "--runs") runs = std::atoi(next());
        else if (a == "--method") {
            std::string m = next();
            if (m != "basic") {
                std::fprintf(stderr, "--method %s: only the basic renderer is on the device path\n", m.c_str());
                return 2;
            }
        } else {
            usage();
            return 2;
        }
    }
    Scene scene;
    if (scene_name == "my_scene") create_scene(scene);
    else if (scene_name == "bench128") create_bench_128_scene(scene);
    else if (scene_name == "synth2" || scene_name == "synth3") {
        rt_synth_params p;
        rt_synth_config(scene_name == "synth2" ? 2 : 3, &p);
        create_synth_scene(scene, p);
    } else {
        usage();
        return 2;
    }
    std::printf("Rendering configuration: w=%u h=%u depth=%u scene=%s\n", w, h, depth, scene_name.c_str());

    auto flat = scene.flatten();
    rt_scene* s = nullptr;
    rt_status st = rt_scene_create(&flat->desc, device, &s);
    if (st != RT_OK) {
        std::fprintf(stderr, "rt_scene_create: %s\n", rt_status_str(st));
        return 1;
    }
    Camera cam(w, h);
    rt_camera c = cam.to_c();
    std::vector<float> rgb((size_t)w * h * 3);
    std::vector<uint8_t> rgb8((size_t)w * h * 3);
    rt_counters cnt;
    float kms = 0.f;
    rt_render_opts opts{device, &cnt, &kms};
    int n = bench ? runs : 1;
    auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < n; k++) {
        auto r0 = std::chrono::steady_clock::now();
        st = rt_render(s, &c, depth, &opts, rgb.data(), rgb8.data());
        if (st != RT_OK) {
            std::fprintf(stderr, "rt_render: %s\n", rt_status_str(st));
            return 1;
        }
        auto r1 = std::chrono::steady_clock::now();
        std::printf("render_scene: %lldms (kernel %.3f ms)\n",
                    (long long)std::chrono::duration_cast<std::chrono::milliseconds>(r1 - r0).count(), kms);
    }
    auto t1 = std::chrono::steady_clock::now();
    if (bench) {
        long long ns = (long long)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
        std::printf("Total Time: %lldms | %lldns\n", ns / 1000000, ns);
        std::printf("Avg Per Op: %gms | %gns\n", (double)ns / 1e6 / n, (double)ns / n);
    }
    std::printf("rays: node %llu shadow %llu pixels %llu\n", (unsigned long long)cnt.node_rays,
                (unsigned long long)cnt.shadow_rays, (unsigned long long)cnt.pixels);
    if (!out.empty()) {
        bool ok = out.size() > 4 && out.substr(out.size() - 4) == ".ppm" ? write_ppm(out, rgb8, w, h)
                                                                          : write_bmp(out, rgb8, w, h);
        if (!ok) {
            std::fprintf(stderr, "cannot write %s\n", out.c_str());
            return 1;
        }
        std::printf("wrote %s\n", out.c_str());
    }
    rt_scene_destroy(s);
    return 0;
}
