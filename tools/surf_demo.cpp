// surf_demo.cpp -- the reference's main.cpp flow (cudaSurfDemo2,
// main.cpp:163-283) against this engine's drop-in headers, minus OpenCV:
// images come from a PGM reader instead of cv::imread and nothing is drawn.
// Usage: surf_demo [device] [left.pgm] [right.pgm] [repeats] [dump_prefix]
// With dump_prefix, writes <prefix>_left.bin / _right.bin (after detection)
// and <prefix>_match.bin (set 1 after match): int32 n, int32 nfeatures, then
// n SurfPoints (h_data) and n x nfeatures descriptor floats (none in _match).
#include <cstdio>
#include <memory>
#include <vector>

#include "surf.h"

extern "C" long surf_pgm_info(const char* path, int* w, int* h);
extern "C" int surf_pgm_read(const char* path, unsigned char* dst, int pitch);

typedef unsigned char uchar;

static bool load(const char* path, std::vector<uchar>& px, int& w, int& h)
{
    if (surf_pgm_info(path, &w, &h) < 0)
        return false;
    px.assign((size_t)w * h, 0);
    return surf_pgm_read(path, px.data(), w) == 0;
}

static bool dump(const char* prefix, const char* tag, const surf::SurfData& d, const float* d_desc, int nf)
{
    char path[1024];
    snprintf(path, sizeof path, "%s_%s.bin", prefix, tag);
    FILE* f = fopen(path, "wb");
    if (!f) return false;
    const int hdr[2] = {d.num_pts, d_desc ? nf : 0};
    bool ok = fwrite(hdr, sizeof hdr, 1, f) == 1;
    if (d.num_pts > 0)
        ok = ok && fwrite(d.h_data, sizeof(surf::SurfPoint), d.num_pts, f) == (size_t)d.num_pts;
    if (d_desc && d.num_pts > 0)
    {
        std::vector<float> h((size_t)d.num_pts * nf);
        CHECK(cudaMemcpy(h.data(), d_desc, h.size() * sizeof(float), cudaMemcpyDeviceToHost));
        ok = ok && fwrite(h.data(), sizeof(float), h.size(), f) == h.size();
    }
    return fclose(f) == 0 && ok;
}

int main(int argc, char** argv)
{
    const int devNum = argc > 1 ? atoi(argv[1]) : 0;
    const char* lpath = argc > 2 ? argv[2] : "data/left.pgm";
    const char* rpath = argc > 3 ? argv[3] : "data/right.pgm";
    const int nrepeats = argc > 4 ? atoi(argv[4]) : 100;
    const char* prefix = argc > 5 ? argv[5] : nullptr;

    std::vector<uchar> limg, rimg;
    int lw, lh, rw, rh;
    if (!load(lpath, limg, lw, lh) || !load(rpath, rimg, rw, rh))
    {
        fprintf(stderr, "cannot read %s / %s\n", lpath, rpath);
        return 1;
    }
    std::cout << "Image size = (" << lw << "," << lh << ")" << std::endl;

    // main.cpp:187-204
    int samplingStep = 2, octaves = 4, initLobe = 3, indexSize = 4, max_npts = 10000;
    float thres = 4.f;
    bool doubleImageSize = false, upright = true, extended = false;

    initDevice(devNum);
    GpuTimer timer(0);
    int3 whp1, whp2;
    whp1.x = lw; whp1.y = lh; whp1.z = iAlignUp(whp1.x, 128);
    whp2.x = rw; whp2.y = rh; whp2.z = iAlignUp(whp2.x, 128);
    uchar* img1 = NULL;
    uchar* img2 = NULL;
    size_t tmp_pitch = 0;
    CHECK(cudaMallocPitch((void**)&img1, &tmp_pitch, sizeof(uchar) * whp1.x, whp1.y));
    CHECK(cudaMallocPitch((void**)&img2, &tmp_pitch, sizeof(uchar) * whp2.x, whp2.y));
    // the engine reads rows at pitch whp.z (iAlignUp(w, 128)), as the reference does
    CHECK(cudaFree(img1));
    CHECK(cudaFree(img2));
    CHECK(cudaMalloc(&img1, (size_t)whp1.z * whp1.y));
    CHECK(cudaMalloc(&img2, (size_t)whp2.z * whp2.y));
    CHECK(cudaMemcpy2D(img1, whp1.z, limg.data(), lw, lw, whp1.y, cudaMemcpyHostToDevice));
    CHECK(cudaMemcpy2D(img2, whp2.z, rimg.data(), rw, rw, whp2.y, cudaMemcpyHostToDevice));
    float t0 = timer.read();

    surf::SurfData surf_data1, surf_data2;
    surf::initSurfData(surf_data1, max_npts, true, true);
    surf::initSurfData(surf_data2, max_npts, true, true);
    float* surf_descriptors1 = NULL;
    float* surf_descriptors2 = NULL;

    std::unique_ptr<surf::Surfor> detector(new surf::Surfor);
    detector->init(octaves, thres, doubleImageSize, initLobe * 3, samplingStep, upright, extended, indexSize, lw, lh);

    float t1 = timer.read();
    for (int i = 0; i < nrepeats; i++)
    {
        if (surf_descriptors1) CHECK(cudaFree(surf_descriptors1));
        if (surf_descriptors2) CHECK(cudaFree(surf_descriptors2));
        detector->detectAndCompute(img1, surf_data1, whp1, &surf_descriptors1, true);
        detector->detectAndCompute(img2, surf_data2, whp2, &surf_descriptors2, true);
    }
    float t2 = timer.read();
    const int nf = 16 * indexSize * indexSize / 4 * (extended ? 2 : 1);
    if (prefix && !(dump(prefix, "left", surf_data1, surf_descriptors1, nf) &&
                    dump(prefix, "right", surf_data2, surf_descriptors2, nf)))
    {
        fprintf(stderr, "cannot write %s_*.bin\n", prefix);
        return 1;
    }
    // main.cpp:248-251
    for (int i = 0; i < nrepeats; i++)
        detector->match(surf_data1, surf_data2, surf_descriptors1, surf_descriptors2);
    float t3 = timer.read();
    if (prefix && !dump(prefix, "match", surf_data1, nullptr, nf))
        return 1;

    std::cout << "Number of features1: " << surf_data1.num_pts << std::endl
              << "Number of features2: " << surf_data2.num_pts << std::endl;
    std::cout << "Time for allocating image memory:  " << t0 << std::endl
              << "Time for allocating point memory:  " << t1 - t0 << std::endl
              << "Time of detection and computation: " << (t2 - t1) / nrepeats << std::endl
              << "Time of matching surf keypoints:   " << (t3 - t2) / nrepeats << std::endl;
    for (int i = 0; i < std::min(3, surf_data1.num_pts); i++)
    {
        const surf::SurfPoint& p = surf_data1.h_data[i];
        printf("kp %d: x=%.4f y=%.4f scale=%.4f o=%d strength=%.4f laplace=%d\n", i, p.x, p.y, p.scale, p.o,
               p.strength, p.laplace);
    }

    surf::freeSurfData(surf_data1);
    surf::freeSurfData(surf_data2);
    CHECK(cudaFree(img1));
    CHECK(cudaFree(img2));
    if (surf_descriptors1) cudaFree(surf_descriptors1);
    if (surf_descriptors2) cudaFree(surf_descriptors2);
    CHECK(cudaDeviceReset());
    return 0;
}
