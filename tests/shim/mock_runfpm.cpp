// mock_runfpm.cpp -- drives include/fpm_shim.hpp (the reference-side runFPM
// binding of INTEGRATION.md) on a mock FPM_Dataset laid out exactly like the
// reference's (fpmMain.h:19-101, fpmMain.cpp:42-57,171):
//   * imageStack has ledCount+1 slots indexed by LED NUMBER, slot 0 a dummy;
//   * every slot starts as the CV_8UC1 Np x Np zero image of fpmMain.cpp:42
//     with garbage crop offsets (the reference leaves them indeterminate);
//   * only LEDs of sortedIndicies[0..ledUsedCount) get a 16-bit image and
//     real cropXStart / cropYStart.
// Test fixture only (tests/test_shim.py); not part of the product.
//
// usage: mock_runfpm <input.bin> <out_dir> [--corrupt]
//   input.bin (little endian): int32 np, L, led_count, n_used, itr;
//     float32 objectiveNA, ps_eff, lambda, delta1, delta2;
//     int16 sorted[n_used], crop_x0[n_used], crop_y0[n_used];
//     uint16 images[n_used][np][np] in sorted order
//   --corrupt: the image of sortedIndicies[3] stays the 8-bit dummy; the shim
//     must refuse it before any device call (exit code 4).
// Writes objF / objCrop / pupil / pupilSupport as complex128 .npy (the
// reference's CV_64FC2 members) and prints the shim's log lines.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "../../include/fpm_shim.hpp"

namespace {

enum { MOCK_8UC1 = 0, MOCK_16UC1 = 2 };  // cv::Mat type codes

struct MockMat {  // stands in for cv::UMat
    int type = MOCK_8UC1, rows = 0, cols = 0;
    std::vector<unsigned char> bytes;
};

struct MockImg {  // FPMimg (fpmMain.h:19-41), the fields runFPM touches
    MockMat Image;
    int16_t cropXStart, cropYStart;
};

struct MockDataset {  // FPM_Dataset (fpmMain.h:43-101), the fields runFPM touches
    int16_t Np, Nlarge, Mlarge, Ncrop;
    float objectiveNA, ps_eff, lambda, delta1, delta2;
    float eps = 0.0000000001;
    int16_t itrCount;
    uint16_t ledCount, ledUsedCount;
    std::vector<int16_t> sortedIndicies;
    std::vector<MockImg> imageStack;
    std::vector<double> objF, objCrop, pupil, pupilSupport;  // CV_64FC2
};

template <class T>
bool rd(std::ifstream &f, T *v, size_t n = 1) {
    return (bool)f.read(reinterpret_cast<char *>(v), sizeof(T) * n);
}

bool write_npy_c128(const std::string &path, const std::vector<double> &d, int rows, int cols) {
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) return false;
    char dict[128];
    snprintf(dict, sizeof dict, "{'descr': '<c16', 'fortran_order': False, 'shape': (%d, %d), }", rows, cols);
    std::string hdr = dict;
    const size_t pad = (64 - (10 + hdr.size() + 1) % 64) % 64;
    hdr.append(pad, ' ');
    hdr.push_back('\n');
    const unsigned char magic[8] = {0x93, 'N', 'U', 'M', 'P', 'Y', 1, 0};
    const unsigned short hl = (unsigned short)hdr.size();
    fwrite(magic, 1, 8, f);
    fwrite(&hl, 2, 1, f);
    fwrite(hdr.data(), 1, hdr.size(), f);
    fwrite(d.data(), sizeof(double), d.size(), f);
    return fclose(f) == 0;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 3) {
        std::cerr << "usage: mock_runfpm <input.bin> <out_dir> [--corrupt]" << std::endl;
        return 2;
    }
    const bool corrupt = argc > 3 && std::string(argv[3]) == "--corrupt";
    std::ifstream f(argv[1], std::ios::binary);
    int32_t hdr[5];
    float fl[5];
    if (!rd(f, hdr, 5) || !rd(f, fl, 5)) {
        std::cerr << "bad input header" << std::endl;
        return 2;
    }
    const int np = hdr[0], L = hdr[1], led_count = hdr[2], n_used = hdr[3];
    MockDataset d;
    d.Np = d.Ncrop = (int16_t)np;
    d.Nlarge = d.Mlarge = (int16_t)L;
    d.ledCount = (uint16_t)led_count;
    d.ledUsedCount = (uint16_t)n_used;
    d.itrCount = (int16_t)hdr[4];
    d.objectiveNA = fl[0];
    d.ps_eff = fl[1];
    d.lambda = fl[2];
    d.delta1 = fl[3];
    d.delta2 = fl[4];
    std::vector<int16_t> cx(n_used), cy(n_used);
    d.sortedIndicies.resize(n_used);
    if (!rd(f, d.sortedIndicies.data(), n_used) || !rd(f, cx.data(), n_used) || !rd(f, cy.data(), n_used)) {
        std::cerr << "bad input tables" << std::endl;
        return 2;
    }
    // fpmMain.cpp:42,52-57: ledCount+1 copies of the 8-bit dummy, crops never set
    MockImg dummy;
    dummy.Image.type = MOCK_8UC1;
    dummy.Image.rows = dummy.Image.cols = np;
    dummy.Image.bytes.assign((size_t)np * np, 0);
    dummy.cropXStart = dummy.cropYStart = (int16_t)0x5A5A;
    d.imageStack.assign((size_t)led_count + 1, dummy);
    for (int i = 0; i < n_used; ++i) {  // fpmMain.cpp:171: imageStack.at(led_num) = currentImage
        MockImg img;
        img.Image.type = MOCK_16UC1;
        img.Image.rows = img.Image.cols = np;
        img.Image.bytes.resize((size_t)np * np * 2);
        if (!rd(f, img.Image.bytes.data(), img.Image.bytes.size())) {
            std::cerr << "bad input images" << std::endl;
            return 2;
        }
        img.cropXStart = cx[i];
        img.cropYStart = cy[i];
        if (corrupt && i == 3) continue;  // slot keeps the 8-bit dummy
        d.imageStack.at(d.sortedIndicies[i]) = img;
    }
    std::cout << "naRadius " << fpm_shim::na_radius(&d) << std::endl;

    auto copy_image = [](const MockImg &slot, uint16_t *dst, int n) {
        if (slot.Image.type != MOCK_16UC1 || slot.Image.rows != n || slot.Image.cols != n) return false;
        std::memcpy(dst, slot.Image.bytes.data(), (size_t)n * n * 2);
        return true;
    };
    auto store = [&d](const float *objF, const float *objCrop, const float *pupil, const float *support, int Lr,
                      int n) {  // CV_32FC2 -> CV_64FC2 (convertTo in the OpenCV adapter)
        d.objF.assign(objF, objF + 2 * (size_t)Lr * Lr);
        d.objCrop.assign(objCrop, objCrop + 2 * (size_t)Lr * Lr);
        d.pupil.assign(pupil, pupil + 2 * (size_t)n * n);
        d.pupilSupport.assign(2 * (size_t)n * n, 0.0);
        for (size_t k = 0; k < (size_t)n * n; ++k) d.pupilSupport[2 * k] = support[k];
    };
    const int rc = fpm_shim::runFPM(&d, copy_image, store, std::cout);
    if (rc != FPM_OK) {
        std::cout << "shim rc " << rc << std::endl;
        return rc == FPM_ERR_INVAL ? 4 : 1;
    }
    const std::string o = argv[2];
    const bool ok = write_npy_c128(o + "/objF.npy", d.objF, L, L) && write_npy_c128(o + "/objCrop.npy", d.objCrop, L, L) &&
                    write_npy_c128(o + "/pupil.npy", d.pupil, np, np) &&
                    write_npy_c128(o + "/pupilSupport.npy", d.pupilSupport, np, np);
    return ok ? 0 : 1;
}
