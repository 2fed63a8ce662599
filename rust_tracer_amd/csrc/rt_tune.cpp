// rt_tune.cpp -- parser of the tuning strings of rt_tune.hpp.
#include "rt_tune.hpp"

#include <cstdlib>
#include <cstring>
#include <string>

namespace {

bool parse_int(const std::string& v, long long lo, long long hi, long long* out) {
    if (v.empty()) return false;
    char* end = nullptr;
    const long long x = std::strtoll(v.c_str(), &end, 0);
    if (*end != '\0' || x < lo || x > hi) return false;
    *out = x;
    return true;
}

bool parse_real(const std::string& v, double lo, double hi, double* out) {
    if (v.empty()) return false;
    char* end = nullptr;
    const double x = std::strtod(v.c_str(), &end);
    if (*end != '\0' || !(x >= lo && x <= hi)) return false;
    *out = x;
    return true;
}

template <class T>
bool set_int(const std::string& v, long long lo, long long hi, T& field) {
    long long x = 0;
    if (!parse_int(v, lo, hi, &x)) return false;
    field = (T)x;
    return true;
}

// one of names[i] -> values[i], else an integer in [lo, hi]
bool set_named(const std::string& v, const char* const* names, const int* values, int n, int lo, int hi, int& field) {
    for (int i = 0; i < n; i++)
        if (v == names[i]) {
            field = values[i];
            return true;
        }
    return set_int(v, lo, hi, field);
}

bool apply_one(Tune& t, const std::string& k, const std::string& v, bool build) {
    // ---- scene build
    if (k == "bvh" || k == "graze_k" || k == "graze_res" || k == "graze_lane" || k == "lb_res" || k == "lb_reach" ||
        k == "shape_buf" || k == "bvh_tris" || k == "dark_skip" || k == "bvh_cnode" || k == "bvh_maxleaf" ||
        k == "force_rccl" || k == "lb_tiers" || k == "lb_dmax_k" || k == "lb_near_all" || k == "build_threads") {
        if (!build) return false;
        if (k == "bvh") return set_int(v, 0, 1, t.bvh);
        if (k == "graze_k") return parse_real(v, 1e-6, 1.0, &t.graze_k);
        if (k == "graze_res") return set_int(v, 0, 256, t.graze_res);
        if (k == "graze_lane") return set_int(v, 0, 1, t.graze_lane);
        if (k == "lb_res") return set_int(v, 0, 1024, t.lb_res);
        if (k == "lb_reach") return set_int(v, 0, 1, t.lb_reach);
        if (k == "lb_tiers") return set_int(v, 1, 7, t.lb_tiers);
        if (k == "lb_dmax_k") return parse_real(v, 1.0, 100.0, &t.lb_dmax_k);
        if (k == "lb_near_all") return set_int(v, 0, 1, t.lb_near_all);
        if (k == "build_threads") return set_int(v, 0, 256, t.build_threads);
        if (k == "shape_buf") return set_int(v, 0, 1, t.shape_buf);
        if (k == "bvh_tris") return set_int(v, 0, 1, t.bvh_tris);
        if (k == "dark_skip") return set_int(v, 0, 1, t.dark_skip);
        if (k == "bvh_cnode") return parse_real(v, 1.0, 1e6, &t.bvh_cnode);
        if (k == "bvh_maxleaf") return set_int(v, 1, 64, t.bvh_maxleaf);
        return set_int(v, 0, 1, t.force_rccl);
    }
    // ---- per pass
    if (k == "sort") {  // all | shadow | none
        if (v == "all" || v == "1") t.sort_tasks = t.sort_shadow = 1;
        else if (v == "shadow") t.sort_tasks = 0, t.sort_shadow = 1;
        else if (v == "none" || v == "0") t.sort_tasks = t.sort_shadow = 0;
        else return false;
        return true;
    }
    if (k == "sort_shadow") return set_int(v, 0, 1, t.sort_shadow);
    if (k == "task_key") return set_int(v, 0, 7, t.task_key);
    if (k == "self_shadow") return set_int(v, 0, 1, t.self_shadow);
    if (k == "inline_shadow") return set_int(v, 0, 1024, t.inline_shadow);
    if (k == "sched") return set_int(v, 0, 2, t.sched);
    if (k == "task_w") {
        if (!set_int(v, 16, 64, t.task_w)) return false;
        return t.task_w == 16 || t.task_w == 32 || t.task_w == 64;
    }
    if (k == "task_fill") return parse_real(v, 0.0, 1e6, &t.task_fill);
    if (k == "shadow_key") {
        static const char* const n[] = {"cell", "cell2"};
        static const int x[] = {1, 2};
        if (!set_named(v, n, x, 2, 16, 21, t.shadow_key)) return false;
        return t.shadow_key == 1 || t.shadow_key == 2 || t.shadow_key == 16 || t.shadow_key == 18 ||
               t.shadow_key == 21;
    }
    if (k == "walk_linear") return parse_real(v, 0.0, 1e6, &t.walk_linear);
    if (k == "walk_first") return set_int(v, 0, 1, t.walk_first);
    if (k == "task_fine") return set_int(v, 0, 1, t.task_fine);
    if (k == "shadow_fine") return set_int(v, 0, 1, t.shadow_fine);
    if (k == "key24") return set_int(v, 0, 1, t.key24);
    if (k == "spp_keys" || k == "frame_keys") {
        static const char* const n[] = {"mix", "mixfine", "frame"};
        static const int x[] = {0, 1, 2};
        return set_named(v, n, x, 3, 0, 2, k == "spp_keys" ? t.spp_keys : t.frame_keys);
    }
    if (k == "l0_interleave") return set_int(v, 0, 1, t.l0_interleave);
    if (k == "spp_batch") return set_int(v, 0, 1024, t.spp_batch);
    if (k == "spp_batch_items") return set_int(v, 1, 1ll << 30, t.spp_batch_items);
    if (k == "node_factor") return set_int(v, 2, 1 << 20, t.node_factor);
    if (k == "shadow_factor") return parse_real(v, 0.25, 64.0, &t.shadow_factor);
    if (k == "node_cap") return set_int(v, 0, 1ll << 32, t.node_cap);
    if (k == "grid_pct") return set_int(v, 0, 100, t.grid_pct);
    if (k == "grid_pct_shadow") return set_int(v, 1, 100, t.grid_pct_shadow);
    if (k == "grid_pct_combine") return set_int(v, 1, 100, t.grid_pct_combine);
    if (k == "lds_nodes") {
        static const char* const n[] = {"trace", "shadow", "both"};
        static const int x[] = {1, 2, 3};
        return set_named(v, n, x, 3, 0, 3, t.lds_nodes);
    }
    if (k == "deep_kernel") return set_int(v, 0, 1, t.deep_kernel);
    if (k == "occ_each") return set_int(v, 0, 1, t.occ_each);
    if (k == "count") {
        static const char* const n[] = {"trace", "shadow", "all"};
        static const int x[] = {1, 2, 3};
        return set_named(v, n, x, 3, 1, 3, t.count);
    }
    if (k == "dup") {  // letters s (sorts), h (shadow pass), c (combines)
        int m = 0;
        for (char c : v) {
            if (c == 's') m |= 1;
            else if (c == 'h') m |= 2;
            else if (c == 'c') m |= 4;
            else if (c != '0') return false;
        }
        t.dup = m;
        return true;
    }
    if (k == "seam_split") return set_int(v, 1, 8, t.seam_split);
    if (k == "seam_band_rows") return set_int(v, 0, 1 << 20, t.seam_band_rows);
    if (k == "seam_adapt") {
        static const char* const n[] = {"device"};
        static const int x[] = {2};
        return set_named(v, n, x, 1, 0, 2, t.seam_adapt);
    }
    if (k == "seam_grid_pct") return set_int(v, 1, 100, t.seam_grid_pct);
    if (k == "frame_fork") {
        static const char* const n[] = {"fork", "caller"};
        static const int x[] = {0, 1};
        return set_named(v, n, x, 2, 0, 1, t.frame_fork);
    }
    return false;
}

}  // namespace

bool tune_apply(Tune& t, const char* spec, bool build_keys) {
    if (!spec) return true;
    std::string s(spec);
    size_t i = 0;
    while (i < s.size()) {
        while (i < s.size() && (s[i] == ',' || s[i] == ' ' || s[i] == '\t' || s[i] == '\n')) i++;
        if (i >= s.size()) break;
        size_t j = i;
        while (j < s.size() && s[j] != ',' && s[j] != ' ' && s[j] != '\t' && s[j] != '\n') j++;
        const std::string kv = s.substr(i, j - i);
        i = j;
        const size_t eq = kv.find('=');
        if (eq == std::string::npos || eq == 0) return false;
        if (!apply_one(t, kv.substr(0, eq), kv.substr(eq + 1), build_keys)) return false;
    }
    return true;
}
