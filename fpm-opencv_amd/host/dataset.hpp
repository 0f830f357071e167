// dataset.hpp -- host-side mirror of the reference's FPM_Dataset, its JSON
// contract (fpmMain.cpp:508-587), LED geometry (fpmMain.cpp:59-106,146-168),
// LED order (fpmMain.cpp:246-258 + fpmMain.h:103-115) and image
// pre-processing (fpmMain.cpp:109-144).  Arithmetic keeps the reference's
// float/double/int16 types so crop offsets and the tie order of std::sort come
// out identical.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "json.hpp"

namespace fpmhost {

struct Config {
    // fpmMain.cpp:517-575, in that order, with the same defaults
    std::string file_prefix = "iLED_";
    std::string file_extension = ".tif";
    int16_t np = 90;
    std::string dataset_root = ".";
    float pixel_size = 6.5f;
    float objective_mag = 8.f;
    float objective_na = 0.2f;
    float max_illumination_na = 0.7604f;
    bool color = false;
    int16_t center_led = 249;
    float lambda = 0.5f;
    float ps_eff = 0.f;
    float du = 0.f;
    bool leading_zeros = false;
    int16_t crop_x = 1, crop_y = 1;
    double array_rotation = 0.0;
    int16_t bk1_crop_x = 1, bk1_crop_y = 1, bk2_crop_x = 1, bk2_crop_y = 1;
    int16_t hole_number_digits = 4;
    int16_t res_improvement_factor = 1;
    float bg_threshold = 1000.f;
    int16_t mcrop = 0, ncrop = 0, nlarge = 0, mlarge = 0;
    float ps = 0.f;
    float delta1 = 5.f, delta2 = 10.f;
    uint16_t led_count = 508;
    bool flip_x = false, flip_y = false;
    uint16_t darkfield_exp_multiplier = 1;
    std::string hole_coordinate_file = "null";
    bool debug = false;
    // derived for runFPM (fpmMain.cpp:305-306)
    int16_t na_radius = 0;
    // source of LED coordinates
    Json hole_coordinates;           // datasetJson.get("holeCoordinates", 0)
    bool hole_coordinates_array = false;
    bool json_ok = true;             // Json::Reader::parse result (ignored by the reference)
    std::string json_error;
};

// Parse a dataset JSON exactly as main() does. A missing/unreadable file
// yields all defaults (the reference ignores the ifstream state too).
Config load_config(const std::string &json_path);
Config config_from_text(const std::string &text);
Config config_from_json(const JsonParseResult &parsed);

struct LedGeom {
    int led = 0;              // LED number (1-based, as in the file name)
    float pos[3] = {0, 0, 0}; // holeCoordinates[led-1] x, y, z (asFloat)
    double sin_x = 0, sin_y = 0;
    float na = 0;             // illumination_na
    bool used = false;        // NA < maxIlluminationNA (fpmMain.cpp:106)
    float uled = 0, vled = 0;
    int16_t idx_u = 0, idx_v = 0;
    int16_t crop_x0 = 0, crop_y0 = 0;   // cropXStart / cropYStart
    int16_t crop_x1 = 0, crop_y1 = 0;   // cropXEnd / cropYEnd
};

// LED coordinate provider: holeCoordinates from the JSON, or an explicit
// table (e.g. the 508-LED dome, used when the JSON has none -- SURVEY 8(c)).
struct LedTable {
    std::vector<float> xyz;   // [n][3]
    int n() const { return (int)(xyz.size() / 3); }
};

// Geometry of every LED number in `present` (images found on disk).
// Throws std::runtime_error where the reference would abort (no coordinate
// table at all, LED number > ledCount).
std::vector<LedGeom> compute_geometry(const Config &cfg, const std::vector<int> &present,
                                      const LedTable *override_table);

// sortedIndicies (fpmMain.cpp:246-258): std::sort of the ledCount+1 NA list
// (99.0 for LEDs without an image), first ledUsedCount entries.
std::vector<int16_t> sorted_indices(const Config &cfg, const std::vector<LedGeom> &geoms);

// Directory scan (fpmMain.cpp:63-75): LED numbers of files named
// <prefix><N><ext> in datasetRoot; the file name per LED is also returned.
int scan_dataset(const Config &cfg, std::vector<int> *leds, std::vector<std::string> *names,
                 std::string *err);

// Pre-processing of one full frame (fpmMain.cpp:124-144): Np x Np crop at
// (cropX, cropY), darkfield divide, background = mean of two Np x Np windows
// clamped to bgThresh and rounded, saturating subtract.
struct Frame {
    int width = 0, height = 0;
    std::vector<uint16_t> px;  // row-major
};
bool preprocess_frame(const Config &cfg, const Frame &full, float illumination_na, std::vector<uint16_t> *out,
                      int16_t *bg_val, std::string *err);

}  // namespace fpmhost
