// ref_probe.cpp -- TEST INFRASTRUCTURE ONLY (oracle).  Never linked into the
// product.  Built by oracle/Makefile into oracle/_ref/ref_probe, linked with
// the reference's OWN vendored jsoncpp 1.6.5 compiled in place from
// /root/reference/include/jsoncpp.cpp (the only part of the reference that
// builds here: fpmMain.cpp itself needs OpenCV 3 and cvComplex, which are
// absent -- SURVEY.md 8(c)).
//
// It restates main()'s config reads (fpmMain.cpp:512-575) and the loader's
// geometry + LED order (fpmMain.cpp:52-106,146-168,246-258, fpmMain.h:103-115)
// on top of the reference's Json::Value, with the reference's float / double /
// int16 types, and prints one JSON document.  tests/golden/make_golden_geometry.py
// runs it on the shipped dataset JSONs to produce the geometry fixtures that pin
// the product host front-end (libfpm_host.so).
//
// usage: ref_probe <dataset.json> <n_present> [maxIlluminationNA override] [cropSizeX override]
//        LED numbers 1..n_present are treated as present image files.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "json.h"

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: ref_probe dataset.json n_present [maxNA] [cropSizeX]\n");
        return 2;
    }
    Json::Value dj;
    Json::Reader reader;
    std::ifstream jf(argv[1]);
    const bool parse_ok = reader.parse(jf, dj);  // result ignored by the reference (:515)

    // fpmMain.cpp:517-575 -- FPM_Dataset member types from fpmMain.h:43-101
    int16_t Np = dj.get("cropSizeX", 90).asInt();
    float pixelSize = dj.get("pixelSize", 6.5).asDouble();
    float objectiveMag = dj.get("objectiveMag", 8).asDouble();
    float objectiveNA = dj.get("objectiveNA", 0.2).asDouble();
    float maxNA = dj.get("maxIlluminationNA", 0.7604).asDouble();
    float lambda = dj.get("lambda", 0.5).asDouble();
    if (argc > 3) maxNA = (float)atof(argv[3]);
    if (argc > 4) Np = (int16_t)atoi(argv[4]);
    float ps_eff = pixelSize / (float)objectiveMag;
    float du = (1 / ps_eff) / (float)Np;
    double arrayRotation = dj.get("arrayRotation", 0).asInt();
    int16_t rif = 1 + (int16_t)ceil(2 * ps_eff * (maxNA + objectiveNA) / lambda);
    float bgThreshold = dj.get("bgThresh", 1000).asInt();
    int16_t Ncrop = Np, Mcrop = Np;
    int16_t Nlarge = Ncrop * rif, Mlarge = Mcrop * rif;
    float delta1 = dj.get("delta1", 5).asInt();
    float delta2 = dj.get("delta2", 10).asInt();
    uint16_t ledCount = dj.get("ledCount", 508).asInt();
    bool flipX = dj.get("flipDatasetX", false).asBool();
    bool flipY = dj.get("flipDatasetY", false).asBool();
    Json::Value holeCoordinates = dj.get("holeCoordinates", 0);
    int16_t naRadius = (int16_t)ceil(objectiveNA * ps_eff * Np / lambda);  // :305-306

    printf("{\n \"parse_ok\": %s,\n", parse_ok ? "true" : "false");
    printf(" \"np\": %d, \"nlarge\": %d, \"rif\": %d, \"na_radius\": %d,\n", Np, Nlarge, rif, naRadius);
    printf(" \"ps_eff\": %.9g, \"du\": %.9g, \"max_na\": %.9g, \"delta1\": %.9g, \"delta2\": %.9g,\n", ps_eff, du,
           maxNA, delta1, delta2);
    printf(" \"bg_threshold\": %.9g, \"led_count\": %d, \"flip_x\": %d, \"flip_y\": %d,\n", bgThreshold, ledCount,
           flipX, flipY);
    printf(" \"hole_coordinates_is_array\": %s, \"hole_coordinates_size\": %u,\n",
           holeCoordinates.isArray() ? "true" : "false", holeCoordinates.isArray() ? holeCoordinates.size() : 0u);
    if (!holeCoordinates.isArray()) {
        printf(" \"error\": \"no holeCoordinates array: the reference throws Json::LogicError here\"\n}\n");
        return 0;
    }

    const int n_present = atoi(argv[2]);
    std::vector<float> naList(ledCount + 1, 99.0f);  // :52-57
    double angle = arrayRotation;                    // :60-61
    double R[3][3] = {{cos(angle * M_PI / 180), -sin(angle * M_PI / 180), 0},
                      {sin(angle * M_PI / 180), cos(angle * M_PI / 180), 0},
                      {0, 0, 1}};
    int used = 0;
    printf(" \"leds\": [\n");
    for (int led = 1; led <= n_present; ++led) {
        float posX = holeCoordinates[led - 1][0].get("x", 0).asFloat();  // :77-79
        float posY = holeCoordinates[led - 1][1].get("y", 0).asFloat();
        float posZ = holeCoordinates[led - 1][2].get("z", 0).asFloat();
        double in[3] = {posX, posY, posZ}, hc[3];
        for (int j = 0; j < 3; ++j) {
            double s = 0;
            for (int k = 0; k < 3; ++k) s += in[k] * R[k][j];
            hc[j] = s;
        }
        double flip[3] = {1, 1, 1};
        if (flipX) flip[0] = -1, flip[1] = 1;
        if (flipY) flip[0] = 1, flip[1] = -1;
        for (int j = 0; j < 3; ++j) hc[j] *= flip[j];
        double sx = sin(atan2(hc[0], hc[2])), sy = sin(atan2(hc[1], hc[2]));  // :95-99
        float na = sqrt(sx * sx + sy * sy);                                    // :101-103
        int cx0 = 0, cy0 = 0, iu = 0, iv = 0;
        bool is_used = sqrt(na < maxNA);                                        // :106
        if (is_used) {
            float uled = sx / lambda, vled = sy / lambda;                       // :146-147
            int16_t idx_u = (int16_t)round(uled / du), idx_v = (int16_t)round(vled / du);
            int16_t x0 = (int16_t)round(Nlarge / 2) + idx_u - (int16_t)round(Ncrop / 2);  // :157-159
            int16_t y0 = (int16_t)round(Mlarge / 2) + idx_v - (int16_t)round(Ncrop / 2);  // :163-165
            cx0 = x0;
            cy0 = y0;
            iu = idx_u;
            iv = idx_v;
            naList.at(led) = na;
            ++used;
        }
        printf("  {\"led\": %d, \"x\": %.9g, \"y\": %.9g, \"z\": %.9g, \"na\": %.9g, \"used\": %d, \"idx_u\": %d, "
               "\"idx_v\": %d, \"crop_x0\": %d, \"crop_y0\": %d}%s\n",
               led, posX, posY, posZ, na, is_used ? 1 : 0, iu, iv, cx0, cy0, led < n_present ? "," : "");
    }
    printf(" ],\n");
    // fpmMain.h:103-115 + fpmMain.cpp:246-258
    std::vector<size_t> idx(naList.size());
    for (size_t i = 0; i != idx.size(); ++i) idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&naList](size_t i1, size_t i2) { return naList[i1] < naList[i2]; });
    printf(" \"led_used_count\": %d,\n \"sorted_indices\": [", used);
    int incr = 1;
    bool first = true;
    for (size_t i : idx) {
        if (incr <= used) {
            printf("%s%d", first ? "" : ", ", (int)(int16_t)i);
            first = false;
            ++incr;
        }
    }
    printf("]\n}\n");
    return 0;
}
