// fpmMain.cpp -- command-line drop-in for the reference's fpmMain
// (fpmMain.cpp:500-592):  `source use_gpu.sh; fpmMain <dataset.json> <itrCount>`
//
// Same JSON keys and defaults, same argv contract (argc < 3 prints usage and
// returns 0), same log lines ("Dataset Root: ...", "resImprovementFactor: N",
// "Loading Images...", "Loaded: <file>, LED # is: N", "Skipped LED# N",
// "Iteration i Completed (Time: t sec)", "FP Processing Completed (Time: t
// sec)").  The solver runs on the MI355X through libfpm_hip.so.  Instead of
// the reference's blocking showComplexImg windows (fpmMain.cpp:495-497) the
// results are written as .npy files: objCrop (L x L complex64), objF
// (un-centred spectrum), pupil (centred, Np x Np complex64), plus a
// result.json sidecar (geometry, LED order, iterations, timing).
//
// Extra options (after the two positional arguments):
//   --out DIR          output directory (default ".")
//   --device N         GPU ordinal (default 0)
//   --led-table FILE   "x y z" per line, metres or any unit, 1 row per LED:
//                      used when the JSON has no holeCoordinates (the
//                      reference aborts there; SURVEY.md 8(c) dome fallback)
//   --path general|fused|auto
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "../../include/fpm_hip.h"
#include "../../include/fpm_host.h"

namespace {

bool write_npy_c64(const std::string &path, const float *data, int rows, int cols) {
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) return false;
    char dict[128];
    snprintf(dict, sizeof dict, "{'descr': '<c8', 'fortran_order': False, 'shape': (%d, %d), }", rows, cols);
    std::string hdr = dict;
    size_t total = 10 + hdr.size() + 1;
    size_t pad = (64 - total % 64) % 64;
    hdr.append(pad, ' ');
    hdr.push_back('\n');
    const unsigned char magic[8] = {0x93, 'N', 'U', 'M', 'P', 'Y', 1, 0};
    fwrite(magic, 1, 8, f);
    const unsigned short hl = (unsigned short)hdr.size();
    fwrite(&hl, 2, 1, f);
    fwrite(hdr.data(), 1, hdr.size(), f);
    fwrite(data, sizeof(float) * 2, (size_t)rows * cols, f);
    fclose(f);
    return true;
}

bool read_led_table(const std::string &path, std::vector<float> *xyz) {
    std::ifstream f(path);
    if (!f) return false;
    float a, b, c;
    while (f >> a >> b >> c) {
        xyz->push_back(a);
        xyz->push_back(b);
        xyz->push_back(c);
    }
    return !xyz->empty();
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 3) {
        std::cout << "ERROR: Not enough input argumants.\n Usage: ./fpmMain dataset.json" << std::endl;
        return 0;
    }
    std::string out_dir = ".", led_table, path_opt = "auto";
    int device = 0;
    for (int i = 3; i < argc; ++i) {
        std::string a = argv[i];
        if (a == "--out" && i + 1 < argc) out_dir = argv[++i];
        else if (a == "--device" && i + 1 < argc) device = atoi(argv[++i]);
        else if (a == "--led-table" && i + 1 < argc) led_table = argv[++i];
        else if (a == "--path" && i + 1 < argc) path_opt = argv[++i];
        else {
            std::cerr << "unknown option " << a << std::endl;
            return 2;
        }
    }
    // use_cpu.sh / use_gpu.sh select the OpenCL device (use_gpu.sh:1)
    const char *dev = getenv("OPENCV_OPENCL_DEVICE");
    if (dev && strncmp(dev, "CPU", 3) == 0) {
        std::cerr << "OPENCV_OPENCL_DEVICE=" << dev
                  << ": this build runs the solver on MI355X only (source use_gpu.sh). The CPU "
                     "restatement of runFPM lives in oracle/ and is a test checker, not a product path."
                  << std::endl;
        return 3;
    }

    fpm_host *h = nullptr;
    if (fpm_host_open(argv[1], &h)) {
        std::cerr << fpm_host_last_error() << std::endl;
        return 1;
    }
    fpm_host_config cfg;
    fpm_host_get_config(h, &cfg);
    const int itr_count = atoi(argv[2]);  // fpmMain.cpp:569
    std::cout << "Dataset Root: " << cfg.dataset_root << std::endl;
    std::cout << "resImprovementFactor: " << cfg.res_improvement_factor << std::endl;
    if (!led_table.empty()) {
        std::vector<float> xyz;
        if (!read_led_table(led_table, &xyz)) {
            std::cerr << "cannot read LED table " << led_table << std::endl;
            return 1;
        }
        fpm_host_set_led_table(h, xyz.data(), (int)(xyz.size() / 3));
    }
    std::cout << "Loading Images..." << std::endl;
    if (fpm_host_scan(h) < 0) {
        std::cout << "ERROR: Could not Open Directory." << std::endl;
        return 1;
    }
    const int used = fpm_host_geometry(h);
    if (used <= 0) {
        std::cout << fpm_host_last_error() << std::endl;
        return 1;
    }
    std::vector<fpm_host_led> leds(fpm_host_n_present(h));
    fpm_host_get_leds(h, leds.data(), (int)leds.size());
    for (auto &l : leds) {
        std::cout << "NA:" << l.illumination_na << std::endl;
        if (!l.used) std::cout << "Skipped LED# " << l.led << std::endl;
    }
    if (fpm_host_load_images(h) < 0) {
        std::cerr << fpm_host_last_error() << std::endl;
        return 1;
    }
    std::vector<int32_t> order(used), x0(used), y0(used);
    fpm_host_get_order(h, order.data(), used);
    fpm_host_get_crops(h, x0.data(), y0.data(), used);
    for (int i = 0; i < used; ++i) std::cout << "Loaded: LED # is: " << order[i] << std::endl;
    const int np = cfg.np, L = cfg.nlarge;
    std::vector<uint16_t> stack((size_t)used * np * np);
    fpm_host_get_stack(h, stack.data(), stack.size());

    std::vector<int32_t> ident(used);
    for (int i = 0; i < used; ++i) ident[i] = i;  // stack index i == sortedIndicies[i]
    fpm_problem p;
    std::memset(&p, 0, sizeof p);
    p.np = np;
    p.nlarge = L;
    p.n_stack = used;
    p.n_order = used;
    p.order = ident.data();
    p.crop_x0 = x0.data();
    p.crop_y0 = y0.data();
    p.na_radius = cfg.na_radius;
    p.init_pos = 1;
    p.delta1 = cfg.delta1;
    p.delta2 = cfg.delta2;
    p.eps = (double)1e-10f;
    p.n_patch = 1;
    p.path = path_opt == "general" ? FPM_PATH_GENERAL : path_opt == "fused" ? FPM_PATH_FUSED : FPM_PATH_AUTO;
    fpm_ctx *ctx = nullptr;
    int rc = fpm_create(&p, device, &ctx);
    if (!rc) rc = fpm_upload_stack(ctx, stack.data());
    if (!rc) rc = fpm_init(ctx);
    if (rc) {
        std::cerr << "fpm: " << fpm_last_error() << std::endl;
        return 1;
    }
    auto t_all = std::chrono::steady_clock::now();
    for (int itr = 1; itr <= itr_count; ++itr) {
        auto t0 = std::chrono::steady_clock::now();
        if ((rc = fpm_run(ctx, 1))) {
            std::cerr << "fpm: " << fpm_last_error() << std::endl;
            return 1;
        }
        double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::cout << "Iteration " << itr << " Completed (Time: " << dt << " sec)" << std::endl;
    }
    double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_all).count();
    std::cout << "FP Processing Completed (Time: " << dt << " sec)" << std::endl;

    std::vector<float> objF((size_t)L * L * 2), objCrop((size_t)L * L * 2), pupil((size_t)np * np * 2);
    if ((rc = fpm_download(ctx, objF.data(), objCrop.data(), pupil.data(), nullptr))) {
        std::cerr << "fpm: " << fpm_last_error() << std::endl;
        return 1;
    }
    fpm_info info;
    fpm_get_info(ctx, &info);
    fpm_destroy(ctx);
    fpm_host_close(h);
    bool ok = write_npy_c64(out_dir + "/objCrop.npy", objCrop.data(), L, L) &&
              write_npy_c64(out_dir + "/objF.npy", objF.data(), L, L) &&
              write_npy_c64(out_dir + "/pupil.npy", pupil.data(), np, np);
    if (ok) {  // JSON sidecar describing the arrays (replaces the reference's display windows)
        FILE *f = fopen((out_dir + "/result.json").c_str(), "w");
        ok = f != nullptr;
        if (f) {
            fprintf(f, "{\n  \"dataset\": \"%s\",\n  \"iterations\": %d,\n  \"np\": %d,\n  \"nlarge\": %d,\n",
                    argv[1], itr_count, np, L);
            fprintf(f, "  \"na_radius\": %d,\n  \"delta1\": %g,\n  \"delta2\": %g,\n  \"leds_used\": %d,\n",
                    cfg.na_radius, cfg.delta1, cfg.delta2, used);
            fprintf(f, "  \"path\": \"%s\",\n  \"seconds\": %.6f,\n  \"order\": [",
                    info.path == FPM_PATH_FUSED ? "fused" : "general", dt);
            for (int i = 0; i < used; ++i) fprintf(f, "%s%d", i ? ", " : "", order[i]);
            fprintf(f, "],\n  \"arrays\": {\n");
            fprintf(f, "    \"objCrop.npy\": \"complex64 [Nlarge][Nlarge], IDFT(objF)/Nlarge^2 (fpmMain.cpp:481)\",\n");
            fprintf(f, "    \"objF.npy\": \"complex64 [Nlarge][Nlarge], un-centred object spectrum\",\n");
            fprintf(f, "    \"pupil.npy\": \"complex64 [Np][Np], centred pupil (fpmMain.cpp:496)\"\n  }\n}\n");
            fclose(f);
        }
    }
    if (!ok) {
        std::cerr << "cannot write outputs to " << out_dir << std::endl;
        return 1;
    }
    return 0;
}
