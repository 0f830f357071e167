// dataset.cpp -- see dataset.hpp.
#include "dataset.hpp"

#include <dirent.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <stdexcept>

namespace fpmhost {

Config config_from_text(const std::string &text) {
    JsonParseResult pr;
    if (!text.empty()) pr = parse_json(text);
    else {
        pr.ok = false;
        pr.error = "empty document";
    }
    return config_from_json(pr);
}

Config config_from_json(const JsonParseResult &pr) {
    Config c;
    c.json_ok = pr.ok;
    c.json_error = pr.error;
    const Json &j = pr.root;
    auto S = [&](const char *k, const char *d) { return j.get(k, Json::make_string(d)).as_string(); };
    auto I = [&](const char *k, int d) { return j.get(k, Json::make_int(d)).as_int(); };
    auto D = [&](const char *k, double d) { return j.get(k, Json::make_real(d)).as_double(); };
    auto B = [&](const char *k, bool d) { return j.get(k, Json::make_bool(d)).as_bool(); };

    // fpmMain.cpp:517-575 (same order, same defaults, same target types)
    c.file_prefix = S("filePrefix", "iLED_");
    c.file_extension = S("fileExtension", ".tif");
    c.np = (int16_t)I("cropSizeX", 90);
    c.dataset_root = S("datasetRoot", ".");
    c.pixel_size = (float)D("pixelSize", 6.5);
    c.objective_mag = (float)D("objectiveMag", 8);
    c.objective_na = (float)D("objectiveNA", 0.2);
    c.max_illumination_na = (float)D("maxIlluminationNA", 0.7604);
    c.color = B("isColor", false);
    c.center_led = (int16_t)I("centerLED", 249);
    c.lambda = (float)D("lambda", 0.5);
    c.ps_eff = c.pixel_size / (float)c.objective_mag;
    c.du = (1 / c.ps_eff) / (float)c.np;
    c.leading_zeros = B("leadingZeros", false);
    c.crop_x = (int16_t)I("cropX", 1);
    c.crop_y = (int16_t)I("cropY", 1);
    c.array_rotation = (double)I("arrayRotation", 0);
    c.bk1_crop_x = (int16_t)I("bk1cropX", 1);
    c.bk1_crop_y = (int16_t)I("bk1cropY", 1);
    c.bk2_crop_x = (int16_t)I("bk2cropX", 1);
    c.bk2_crop_y = (int16_t)I("bk2cropY", 1);
    c.hole_number_digits = (int16_t)I("holeNumberDigits", 4);
    // fpmMain.cpp:556-558: float arithmetic throughout
    c.res_improvement_factor =
        (int16_t)(1 + (int16_t)std::ceil(2 * c.ps_eff * (c.max_illumination_na + c.objective_na) / c.lambda));
    c.bg_threshold = (float)I("bgThresh", 1000);
    c.mcrop = c.np;
    c.ncrop = c.np;
    c.nlarge = (int16_t)(c.ncrop * c.res_improvement_factor);
    c.mlarge = (int16_t)(c.mcrop * c.res_improvement_factor);
    c.ps = c.ps_eff / (float)c.res_improvement_factor;
    c.delta1 = (float)I("delta1", 5);
    c.delta2 = (float)I("delta2", 10);
    c.led_count = (uint16_t)I("ledCount", 508);
    c.flip_x = B("flipDatasetX", false);
    c.flip_y = B("flipDatasetY", false);
    c.darkfield_exp_multiplier = (uint16_t)I("darkfieldExpMultiplier", 1);
    c.hole_coordinate_file = S("holeCoordinateFileName", "null");
    c.hole_coordinates = j.get("holeCoordinates", Json::make_int(0));
    c.hole_coordinates_array = c.hole_coordinates.is_array();
    c.debug = B("debug", false);
    // naRadius, fpmMain.cpp:305-306 (float products, int16 ceil)
    c.na_radius = (int16_t)std::ceil(c.objective_na * c.ps_eff * c.np / c.lambda);
    return c;
}

Config load_config(const std::string &json_path) {
    std::string text;
    if (!read_file(json_path, &text)) text.clear();
    return config_from_text(text);
}

namespace {

// holeCoordinates[led-1][k].get(key, 0).asFloat() with jsoncpp's non-const
// operator[] semantics (fpmMain.cpp:77-79)
float hole_coord(const Json &hc, int led, int k, const char *key) {
    if (!hc.is_array() && !hc.is_null())
        throw std::runtime_error("in Json::Value::operator[](ArrayIndex): requires arrayValue "
                                 "(the dataset JSON has no holeCoordinates array)");
    if (led - 1 < 0) throw std::runtime_error("in Json::Value::operator[](int index): index cannot be negative");
    const Json &e = hc.at((size_t)(led - 1));
    if (!e.is_array() && !e.is_null())
        throw std::runtime_error("in Json::Value::operator[](ArrayIndex): requires arrayValue");
    const Json &f = e.at((size_t)k);
    if (!f.is_object() && !f.is_null())
        throw std::runtime_error("in Json::Value::find(key, end, found): requires objectValue or nullValue");
    return f.get(key, Json::make_int(0)).as_float();
}

}  // namespace

std::vector<LedGeom> compute_geometry(const Config &cfg, const std::vector<int> &present,
                                      const LedTable *table) {
    std::vector<LedGeom> out;
    // fpmMain.cpp:60-61: rotation about z, angle in degrees (double)
    const double angle = cfg.array_rotation;
    const double R[3][3] = {{std::cos(angle * M_PI / 180), -std::sin(angle * M_PI / 180), 0},
                            {std::sin(angle * M_PI / 180), std::cos(angle * M_PI / 180), 0},
                            {0, 0, 1}};
    for (int led : present) {
        LedGeom g;
        g.led = led;
        if (table) {
            if (led - 1 >= 0 && led - 1 < table->n()) {
                for (int k = 0; k < 3; ++k) g.pos[k] = table->xyz[(size_t)(led - 1) * 3 + k];
            }
        } else {
            g.pos[0] = hole_coord(cfg.hole_coordinates, led, 0, "x");
            g.pos[1] = hole_coord(cfg.hole_coordinates, led, 1, "y");
            g.pos[2] = hole_coord(cfg.hole_coordinates, led, 2, "z");
        }
        // (1x3 double) * Rz, fpmMain.cpp:81-85
        const double in[3] = {g.pos[0], g.pos[1], g.pos[2]};
        double hcrd[3];
        for (int j = 0; j < 3; ++j) {
            double s = 0;
            for (int k = 0; k < 3; ++k) s += in[k] * R[k][j];
            hcrd[j] = s;
        }
        // flips, fpmMain.cpp:88-93 (Y overrides X when both are set)
        double flip[3] = {1, 1, 1};
        if (cfg.flip_x) { flip[0] = -1; flip[1] = 1; flip[2] = 1; }
        if (cfg.flip_y) { flip[0] = 1; flip[1] = -1; flip[2] = 1; }
        for (int j = 0; j < 3; ++j) hcrd[j] *= flip[j];
        // fpmMain.cpp:95-103
        g.sin_x = std::sin(std::atan2(hcrd[0], hcrd[2]));
        g.sin_y = std::sin(std::atan2(hcrd[1], hcrd[2]));
        g.na = (float)std::sqrt(g.sin_x * g.sin_x + g.sin_y * g.sin_y);
        // fpmMain.cpp:106: sqrt(bool) is non-zero iff NA < maxNA
        g.used = g.na < cfg.max_illumination_na;
        if (g.used) {
            if (led > (int)cfg.led_count)
                throw std::runtime_error("LED number " + std::to_string(led) + " exceeds ledCount " +
                                         std::to_string(cfg.led_count) + " (imageStack.at out of range)");
            // fpmMain.cpp:146-168
            g.uled = (float)(g.sin_x / cfg.lambda);
            g.vled = (float)(g.sin_y / cfg.lambda);
            g.idx_u = (int16_t)std::round(g.uled / cfg.du);
            g.idx_v = (int16_t)std::round(g.vled / cfg.du);
            const int16_t half_large_x = (int16_t)std::round(cfg.nlarge / 2);
            const int16_t half_large_y = (int16_t)std::round(cfg.mlarge / 2);
            const int16_t half_crop = (int16_t)std::round(cfg.ncrop / 2);
            g.crop_x0 = (int16_t)(half_large_x + g.idx_u - half_crop);
            g.crop_x1 = (int16_t)(half_large_x + g.idx_u + half_crop - 1);
            g.crop_y0 = (int16_t)(half_large_y + g.idx_v - half_crop);
            g.crop_y1 = (int16_t)(half_large_y + g.idx_v + half_crop - 1);
        }
        out.push_back(g);
    }
    return out;
}

std::vector<int16_t> sorted_indices(const Config &cfg, const std::vector<LedGeom> &geoms) {
    // fpmMain.cpp:52-57: NA list of ledCount+1 entries, 99.0 where no image
    std::vector<float> na((size_t)cfg.led_count + 1, 99.0f);
    int used = 0;
    for (const LedGeom &g : geoms) {
        if (!g.used) continue;
        na.at((size_t)g.led) = g.na;
        ++used;
    }
    // fpmMain.h:103-115: std::sort of indices by NA (not stable)
    std::vector<size_t> idx(na.size());
    for (size_t i = 0; i != idx.size(); ++i) idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&na](size_t i1, size_t i2) { return na[i1] < na[i2]; });
    // fpmMain.cpp:247-258: first ledUsedCount entries
    std::vector<int16_t> out;
    int incr = 1;
    for (size_t i : idx) {
        if (incr <= used) {
            out.push_back((int16_t)i);
            ++incr;
        }
    }
    return out;
}

int scan_dataset(const Config &cfg, std::vector<int> *leds, std::vector<std::string> *names, std::string *err) {
    DIR *dir = opendir(cfg.dataset_root.c_str());
    if (!dir) {
        *err = "ERROR: Could not Open Directory.";
        return -1;
    }
    struct dirent *ent;
    std::vector<std::pair<std::string, int>> found;
    while ((ent = readdir(dir)) != nullptr) {
        std::string fn = ent->d_name;
        const std::string &ext = cfg.file_extension, &pre = cfg.file_prefix;
        // fpmMain.cpp:69-75
        if (fn == "." || fn == "..") continue;
        if (fn.size() < ext.size() || fn.compare(fn.size() - ext.size(), ext.size(), ext) != 0) continue;
        if (fn.find(pre) != 0) continue;
        std::string hole = fn.substr(pre.size(), fn.size() - ext.size() - pre.size());
        found.emplace_back(fn, atoi(hole.c_str()));
    }
    closedir(dir);
    // directory order is unspecified; sort by name for reproducible logs
    std::sort(found.begin(), found.end());
    for (auto &f : found) {
        names->push_back(f.first);
        leds->push_back(f.second);
    }
    return 0;
}

bool preprocess_frame(const Config &cfg, const Frame &full, float illumination_na, std::vector<uint16_t> *out,
                      int16_t *bg_val, std::string *err) {
    const int np = cfg.np;
    auto inside = [&](int x, int y) { return x >= 0 && y >= 0 && x + np <= full.width && y + np <= full.height; };
    if (!inside(cfg.crop_x, cfg.crop_y) || !inside(cfg.bk1_crop_x, cfg.bk1_crop_y) ||
        !inside(cfg.bk2_crop_x, cfg.bk2_crop_y)) {
        *err = "crop or background window outside the image (cv::Rect assertion in the reference)";
        return false;
    }
    out->assign((size_t)np * np, 0);
    // fpmMain.cpp:124-125
    for (int y = 0; y < np; ++y)
        for (int x = 0; x < np; ++x)
            (*out)[(size_t)y * np + x] = full.px[(size_t)(cfg.crop_y + y) * full.width + cfg.crop_x + x];
    // fpmMain.cpp:128-129: darkfield exposure (saturate_cast rounds to nearest even)
    if (cfg.darkfield_exp_multiplier != 1 && illumination_na > cfg.objective_na) {
        for (auto &v : *out) {
            double q = (double)v / (double)cfg.darkfield_exp_multiplier;
            long r = std::lrint(q);
            v = (uint16_t)std::min<long>(65535, std::max<long>(0, r));
        }
    }
    // fpmMain.cpp:131-140: mean of two windows of the UNDIVIDED frame
    auto mean = [&](int x0, int y0) {
        double s = 0;
        for (int y = 0; y < np; ++y)
            for (int x = 0; x < np; ++x) s += full.px[(size_t)(y0 + y) * full.width + x0 + x];
        return s / ((double)np * np);
    };
    double bk1 = mean(cfg.bk1_crop_x, cfg.bk1_crop_y);
    double bk2 = mean(cfg.bk2_crop_x, cfg.bk2_crop_y);
    double bg = (bk2 + bk1) / 2;
    if (bg > cfg.bg_threshold) bg = cfg.bg_threshold;
    *bg_val = (int16_t)std::round(bg);
    // fpmMain.cpp:143-144: saturating subtract
    for (auto &v : *out) {
        int d = (int)v - (int)*bg_val;
        v = (uint16_t)std::min(65535, std::max(0, d));
    }
    return true;
}

}  // namespace fpmhost
