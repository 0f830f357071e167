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
//   --grid GXxGY       reconstruct a GX x GY field of patches instead of the
//                      reference's single crop: patch (i, j) is cut at
//                      (cropX + j*Np, cropY + i*Np) from every full frame on the
//                      GPU (fpm_upload_frames: the loader preprocessing of
//                      fpmMain.cpp:124-144 per patch), all patches are solved in
//                      one batch, and the stitched objCrop field
//                      (GY*Nlarge x GX*Nlarge complex64) is written as
//                      objCrop_field.npy with pupils.npy [B][Np][Np] (SURVEY.md
//                      8(f2)); result.json describes the grid
//
// Device selection: OPENCV_OPENCL_DEVICE (set by use_gpu.sh / use_cpu.sh) is
// read with OpenCV's "<platform>:<type>:<device>" grammar and the scripts'
// literal "GPU:0" / "CPU:0" form: a CPU type anywhere is refused (exit 3; the
// CPU restatement is the oracle, not a product path), a GPU index selects the
// MI355X ordinal; --device overrides it.
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

bool write_npy_c64_3d(const std::string &path, const float *data, int n0, int n1, int n2) {
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) return false;
    char dict[128];
    snprintf(dict, sizeof dict, "{'descr': '<c8', 'fortran_order': False, 'shape': (%d, %d, %d), }", n0, n1, n2);
    std::string hdr = dict;
    size_t pad = (64 - (10 + hdr.size() + 1) % 64) % 64;
    hdr.append(pad, ' ');
    hdr.push_back('\n');
    const unsigned char magic[8] = {0x93, 'N', 'U', 'M', 'P', 'Y', 1, 0};
    fwrite(magic, 1, 8, f);
    const unsigned short hl = (unsigned short)hdr.size();
    fwrite(&hl, 2, 1, f);
    fwrite(hdr.data(), 1, hdr.size(), f);
    fwrite(data, sizeof(float) * 2, (size_t)n0 * n1 * n2, f);
    return fclose(f) == 0;
}

// OPENCV_OPENCL_DEVICE -> (refuse CPU, GPU ordinal).  OpenCV splits the value
// at ':' into platform, device type(s) ('|'-separated) and device name/index;
// use_gpu.sh / use_cpu.sh write "GPU:0" / "CPU:0" (type first).  Returns 3
// for a CPU selection, else 0 and sets *ordinal when an index is given.
int parse_opencl_device(const char *v, int *ordinal) {
    std::vector<std::string> parts;
    std::string cur;
    for (const char *c = v; *c; ++c) {
        if (*c == ':') {
            parts.push_back(cur);
            cur.clear();
        } else {
            cur.push_back((char)toupper((unsigned char)*c));
        }
    }
    parts.push_back(cur);
    auto has_type = [](const std::string &field, const char *t) {
        size_t p = 0;
        while (p <= field.size()) {
            size_t q = field.find('|', p);
            if (q == std::string::npos) q = field.size();
            if (field.compare(p, q - p, t) == 0) return true;
            p = q + 1;
        }
        return false;
    };
    for (size_t i = 0; i < parts.size() && i < 2; ++i)
        if (has_type(parts[i], "CPU")) return 3;
    auto is_num = [](const std::string &x) { return !x.empty() && x.find_first_not_of("0123456789") == std::string::npos; };
    if (parts.size() == 2 && has_type(parts[0], "GPU") && is_num(parts[1])) *ordinal = atoi(parts[1].c_str());
    else if (parts.size() == 3 && is_num(parts[2])) *ordinal = atoi(parts[2].c_str());
    return 0;
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
    int device = 0, device_opt = -1, gx = 0, gy = 0;
    for (int i = 3; i < argc; ++i) {
        std::string a = argv[i];
        if (a == "--out" && i + 1 < argc) out_dir = argv[++i];
        else if (a == "--device" && i + 1 < argc) device_opt = atoi(argv[++i]);
        else if (a == "--led-table" && i + 1 < argc) led_table = argv[++i];
        else if (a == "--path" && i + 1 < argc) path_opt = argv[++i];
        else if (a == "--grid" && i + 1 < argc) {
            if (sscanf(argv[++i], "%dx%d", &gx, &gy) != 2 || gx < 1 || gy < 1) {
                std::cerr << "--grid wants GXxGY, e.g. 16x16" << std::endl;
                return 2;
            }
        } else {
            std::cerr << "unknown option " << a << std::endl;
            return 2;
        }
    }
    // use_cpu.sh / use_gpu.sh select the OpenCL device (use_gpu.sh:1)
    const char *dev = getenv("OPENCV_OPENCL_DEVICE");
    if (dev && *dev) {
        if (parse_opencl_device(dev, &device) == 3) {
            std::cerr << "OPENCV_OPENCL_DEVICE=" << dev
                      << ": this build runs the solver on MI355X only (source use_gpu.sh). The CPU "
                         "restatement of runFPM lives in oracle/ and is a test checker, not a product path."
                      << std::endl;
            return 3;
        }
    }
    if (device_opt >= 0) device = device_opt;
    std::cout << "Device: MI355X ordinal " << device << std::endl;

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
    const int np = cfg.np, L = cfg.nlarge;
    const bool grid = gx > 0;
    const int B = grid ? gx * gy : 1;
    std::vector<int32_t> order(used), x0(used), y0(used);
    fpm_host_get_order(h, order.data(), used);
    fpm_host_get_crops(h, x0.data(), y0.data(), used);
    std::vector<uint16_t> stack, frames;
    int32_t fw = 0, fh = 0;
    if (!grid) {
        if (fpm_host_load_images(h) < 0) {
            std::cerr << fpm_host_last_error() << std::endl;
            return 1;
        }
        stack.resize((size_t)used * np * np);
        fpm_host_get_stack(h, stack.data(), stack.size());
    } else {
        if (fpm_host_load_frames(h, nullptr, 0, &fw, &fh) < 0) {
            std::cerr << fpm_host_last_error() << std::endl;
            return 1;
        }
        frames.resize((size_t)used * fw * fh);
        if (fpm_host_load_frames(h, frames.data(), frames.size(), nullptr, nullptr) < 0) {
            std::cerr << fpm_host_last_error() << std::endl;
            return 1;
        }
    }
    for (int i = 0; i < used; ++i) std::cout << "Loaded: LED # is: " << order[i] << std::endl;

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
    p.n_patch = B;
    p.path = path_opt == "general" ? FPM_PATH_GENERAL : path_opt == "fused" ? FPM_PATH_FUSED : FPM_PATH_AUTO;
    fpm_ctx *ctx = nullptr;
    int rc = fpm_create(&p, device, &ctx);
    std::vector<int16_t> bg(used, 0);
    if (!rc && !grid) rc = fpm_upload_stack(ctx, stack.data());
    if (!rc && grid) {
        // patch (i, j) of the field at (cropX + j Np, cropY + i Np); the
        // darkfield divide applies where illumination NA > objective NA (:128)
        std::vector<int32_t> px(B), py(B);
        for (int i = 0; i < gy; ++i)
            for (int j = 0; j < gx; ++j) {
                px[i * gx + j] = cfg.crop_x + j * np;
                py[i * gx + j] = cfg.crop_y + i * np;
            }
        std::vector<fpm_host_led> all(fpm_host_n_present(h));
        fpm_host_get_leds(h, all.data(), (int)all.size());
        std::vector<uint8_t> dark(used, 0);
        for (int s2 = 0; s2 < used; ++s2)
            for (auto &l : all)
                if (l.led == order[s2]) dark[s2] = l.illumination_na > cfg.objective_na;
        fpm_frames fr;
        std::memset(&fr, 0, sizeof fr);
        fr.height = fh;
        fr.width = fw;
        fr.patch_x0 = px.data();
        fr.patch_y0 = py.data();
        fr.bk1_x = cfg.bk1_crop_x;
        fr.bk1_y = cfg.bk1_crop_y;
        fr.bk2_x = cfg.bk2_crop_x;
        fr.bk2_y = cfg.bk2_crop_y;
        fr.bg_threshold = cfg.bg_threshold;
        fr.darkfield_exp_multiplier = cfg.darkfield_exp_multiplier;
        fr.darkfield = dark.data();
        rc = fpm_upload_frames(ctx, &fr, frames.data(), 0, bg.data());
        frames.clear();
        frames.shrink_to_fit();
    }
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

    std::vector<float> objF(grid ? 0 : (size_t)L * L * 2), objCrop((size_t)B * L * L * 2),
        pupil((size_t)B * np * np * 2);
    if ((rc = fpm_download(ctx, grid ? nullptr : objF.data(), objCrop.data(), pupil.data(), nullptr))) {
        std::cerr << "fpm: " << fpm_last_error() << std::endl;
        return 1;
    }
    fpm_info info;
    fpm_get_info_sized(ctx, &info, sizeof info);
    fpm_destroy(ctx);
    fpm_host_close(h);
    bool ok;
    if (!grid) {
        ok = write_npy_c64(out_dir + "/objCrop.npy", objCrop.data(), L, L) &&
             write_npy_c64(out_dir + "/objF.npy", objF.data(), L, L) &&
             write_npy_c64(out_dir + "/pupil.npy", pupil.data(), np, np);
    } else {
        // stitch: tile b = (i, j) lands at rows i L, columns j L (tiles do not
        // overlap); row-wise copies of L complex values
        const size_t FW = (size_t)gx * L;
        std::vector<float> field((size_t)gy * L * FW * 2);
        for (int b = 0; b < B; ++b) {
            const int i = b / gx, j = b % gx;
            for (int y = 0; y < L; ++y)
                std::memcpy(&field[(((size_t)i * L + y) * FW + (size_t)j * L) * 2],
                            &objCrop[(((size_t)b * L + y) * L) * 2], (size_t)L * 2 * sizeof(float));
        }
        ok = write_npy_c64(out_dir + "/objCrop_field.npy", field.data(), gy * L, gx * L) &&
             write_npy_c64_3d(out_dir + "/pupils.npy", pupil.data(), B, np, np);
    }
    if (ok) {  // JSON sidecar describing the arrays (replaces the reference's display windows)
        FILE *f = fopen((out_dir + "/result.json").c_str(), "w");
        ok = f != nullptr;
        if (f) {
            fprintf(f, "{\n  \"dataset\": \"%s\",\n  \"iterations\": %d,\n  \"np\": %d,\n  \"nlarge\": %d,\n",
                    argv[1], itr_count, np, L);
            fprintf(f, "  \"na_radius\": %d,\n  \"delta1\": %g,\n  \"delta2\": %g,\n  \"leds_used\": %d,\n",
                    cfg.na_radius, cfg.delta1, cfg.delta2, used);
            fprintf(f, "  \"device\": %d,\n  \"path\": \"%s\",\n  \"seconds\": %.6f,\n  \"order\": [", device,
                    info.path == FPM_PATH_FUSED ? "fused" : "general", dt);
            for (int i = 0; i < used; ++i) fprintf(f, "%s%d", i ? ", " : "", order[i]);
            fprintf(f, "],\n");
            if (grid) {
                fprintf(f, "  \"grid\": {\"gx\": %d, \"gy\": %d, \"patches\": %d, \"frame\": [%d, %d], "
                           "\"patch_origin\": [%d, %d], \"patch_step\": %d},\n  \"bg_val\": [",
                        gx, gy, B, fh, fw, cfg.crop_x, cfg.crop_y, np);
                for (int i = 0; i < used; ++i) fprintf(f, "%s%d", i ? ", " : "", bg[i]);
                fprintf(f, "],\n  \"arrays\": {\n");
                fprintf(f, "    \"objCrop_field.npy\": \"complex64 [gy*Nlarge][gx*Nlarge], patch (i, j) = "
                           "IDFT(objF)/Nlarge^2 of the crop at (cropX + j*Np, cropY + i*Np) at rows i*Nlarge, "
                           "columns j*Nlarge\",\n");
                fprintf(f, "    \"pupils.npy\": \"complex64 [gy*gx][Np][Np], centred pupil per patch, row-major "
                           "patch order\"\n  }\n}\n");
            } else {
                fprintf(f, "  \"arrays\": {\n");
                fprintf(f, "    \"objCrop.npy\": \"complex64 [Nlarge][Nlarge], IDFT(objF)/Nlarge^2 (fpmMain.cpp:481)\",\n");
                fprintf(f, "    \"objF.npy\": \"complex64 [Nlarge][Nlarge], un-centred object spectrum\",\n");
                fprintf(f, "    \"pupil.npy\": \"complex64 [Np][Np], centred pupil (fpmMain.cpp:496)\"\n  }\n}\n");
            }
            ok = fclose(f) == 0;
        }
    }
    if (!ok) {
        std::cerr << "cannot write outputs to " << out_dir << std::endl;
        return 1;
    }
    return 0;
}
