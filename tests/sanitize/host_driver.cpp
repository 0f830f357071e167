// Host front-end driver for the ASan/UBSan build (tests/test_host_sanitizers.py):
// runs the JSON reader, geometry, LED order, crops, image loader and TIFF reader
// of libfpm_host's sources on the files named on the command line, including
// malformed ones.  Exit 0 = every call returned (an error code is fine);
// the sanitizers abort the process on any memory or UB fault.
//   host_driver json <file>...    parse + geometry + order + crops (+ images when present)
//   host_driver tiff <file>...    fpm_host_read_tiff into a bounded buffer
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "fpm_host.h"

static int run_json(const char *path) {
    std::ifstream f(path, std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string text = ss.str();
    fpm_host *h = nullptr;
    int rc = fpm_host_open_text(text.c_str(), &h);
    if (rc != 0 || !h) return 0;
    fpm_host_config cfg;
    fpm_host_get_config(h, &cfg);
    if (fpm_host_scan(h) != 0) {
        std::vector<int32_t> leds(300);
        for (int i = 0; i < 300; ++i) leds[i] = i + 1;
        fpm_host_set_present(h, leds.data(), 300);
    }
    if (fpm_host_geometry(h) == 0) {
        const int n = fpm_host_n_used(h);
        if (n > 0) {
            std::vector<int32_t> order(n), x0(n), y0(n);
            std::vector<fpm_host_led> leds(n);
            fpm_host_get_order(h, order.data(), n);
            fpm_host_get_crops(h, x0.data(), y0.data(), n);
            fpm_host_get_leds(h, leds.data(), n);
            if (fpm_host_load_images(h) == 0) {
                std::vector<uint16_t> st((size_t)n * cfg.np * cfg.np);
                fpm_host_get_stack(h, st.data(), st.size());
            }
        }
    }
    fpm_host_close(h);
    return 0;
}

static int run_tiff(const char *path) {
    std::vector<uint16_t> buf(1 << 16);
    int32_t w = 0, hgt = 0;
    fpm_host_read_tiff(path, buf.data(), buf.size(), &w, &hgt);
    return 0;
}

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    for (int i = 2; i < argc; ++i) {
        if (!strcmp(argv[1], "json")) run_json(argv[i]);
        else if (!strcmp(argv[1], "tiff")) run_tiff(argv[i]);
        else return 2;
    }
    printf("host_driver ok %d files\n", argc - 2);
    return 0;
}
