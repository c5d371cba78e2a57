// vr_api_test — a reference-style caller of the vr:: C++ API (include/octvr.hpp), built by build() and
// run by tests/test_gpu_cpp_api.py.  It drives the API the way the reference's own callers do:
//   * apps/octvr/dump.cpp:76-113 — MapperTemplate(out type, out options, w, h), add_input per camera,
//     dump(std::ofstream&)  (no rapidjson here: the JSON-text overloads);
//   * MapperTemplate(std::ifstream&) + vr::Mapper::stitch on GpuMats with a preview_output
//     (mapper.cpp:193-312);
//   * AsyncMultiMapper::New + push / pop of YUV420P host planes (async.cpp:174-193, the vr_map filter);
//   * FastMapper::stitch_nv12 on a template built without ROI (apps/octvr/map.cpp:91-129).
// Usage: vr_api_test DIR   (DIR holds the case written by the test; outputs are written next to it)
#include <cstdio>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "octvr.hpp"

static std::string slurp(const std::string& p) {
    std::ifstream f(p, std::ios::binary);
    if (!f) throw std::runtime_error("cannot read " + p);
    std::stringstream s;
    s << f.rdbuf();
    return s.str();
}
static void spit(const std::string& p, const void* data, size_t n) {
    std::ofstream f(p, std::ios::binary);
    f.write(static_cast<const char*>(data), (std::streamsize)n);
}
static void spit_mat(const std::string& p, const cv::Mat& m) {
    std::ofstream f(p, std::ios::binary);
    for (int r = 0; r < m.rows; r++) f.write(reinterpret_cast<const char*>(m.ptr(r)), (std::streamsize)(m.cols * m.elemSize()));
}

int main(int argc, char** argv) {
    if (argc != 2) {
        fprintf(stderr, "usage: %s DIR\n", argv[0]);
        return 2;
    }
    const std::string d = std::string(argv[1]) + "/";
    try {
        // ---- the case ---------------------------------------------------------------------------
        std::istringstream head(slurp(d + "case.txt"));
        std::string out_type;
        int W = 0, H = 0, n = 0, blend = 0, pw = 0, ph = 0, use_roi = 1;
        head >> out_type >> W >> H >> n >> blend >> pw >> ph >> use_roi;
        const std::string out_opts = slurp(d + "out_opts.json");
        std::vector<std::string> types(n), opts(n);
        std::vector<cv::Size> sizes(n);
        for (int i = 0; i < n; i++) {
            std::istringstream c(slurp(d + "in" + std::to_string(i) + ".txt"));
            c >> types[i] >> sizes[i].width >> sizes[i].height;
            opts[i] = slurp(d + "in" + std::to_string(i) + "_opts.json");
        }
        std::vector<cv::Mat> frames(n);
        for (int i = 0; i < n; i++) {
            frames[i].create(sizes[i].height * 3 / 2, sizes[i].width, CV_8UC1);
            const std::string raw = slurp(d + "frame" + std::to_string(i) + ".yuv");
            if (raw.size() != frames[i].total()) throw std::runtime_error("bad frame size");
            memcpy(frames[i].data, raw.data(), raw.size());
        }

        // ---- apps/octvr/dump.cpp:76-113 -------------------------------------------------------------
        vr::MapperTemplate mt(out_type, out_opts, W, H);
        for (int i = 0; i < n; i++) mt.add_input(types[i], opts[i], false, use_roi != 0);
        {
            std::ofstream of(d + "rig.dat", std::ios::binary);
            mt.dump(of);
        }
        std::cerr << "dumped " << mt.inputs.size() << " inputs, " << mt.out_size.width << "x" << mt.out_size.height
                  << ", seam masks " << mt.seam_masks.size() << std::endl;

        // ---- template copies are independent: the reference copies its Input vectors by value -------
        {
            vr::MapperTemplate a(out_type, out_opts, W, H);
            a.add_input(types[0], opts[0], false, use_roi != 0);
            vr::MapperTemplate b(a);  // copy construction
            vr::MapperTemplate c(out_type, out_opts, W, H);
            c = a;  // copy assignment
            a.add_input(types[n - 1], opts[n - 1], false, use_roi != 0);
            b.add_input(types[0], opts[0], false, use_roi != 0);
            if (a.inputs.size() != 2 || b.inputs.size() != 2 || c.inputs.size() != 1)
                throw std::runtime_error("MapperTemplate copies share their inputs");
            const cv::Rect& r0 = a.inputs[0].roi;
            const cv::Rect& rb = b.inputs[1].roi;
            const cv::Rect& ra = a.inputs[1].roi;
            const cv::Rect& rn = mt.inputs[n - 1].roi;
            if (rb.x != r0.x || rb.y != r0.y || rb.width != r0.width || rb.height != r0.height ||
                ra.x != rn.x || ra.y != rn.y || ra.width != rn.width || ra.height != rn.height)
                throw std::runtime_error("a template copy received another copy's input");
            c.add_input(types[n - 1], opts[n - 1], false, use_roi != 0);
            if (c.inputs.size() != 2 || b.inputs.size() != 2) throw std::runtime_error("copy assignment shares inputs");
            std::cerr << "template copies independent" << std::endl;
        }

        // ---- a template loaded from .dat, vr::Mapper on GpuMats -------------------------------------
        std::ifstream in_dat(d + "rig.dat", std::ios::binary);
        vr::MapperTemplate mt2(in_dat);
        vr::Mapper mapper(mt2, sizes, blend, true);
        std::vector<cv::cuda::GpuMat> gin(n);
        for (int i = 0; i < n; i++) gin[i].upload(frames[i]);
        cv::cuda::GpuMat gout, gprev(ph, pw, CV_8UC3);
        mapper.stitch(gin, gout, gprev);
        cv::Mat out, prev;
        gout.download(out);
        gprev.download(prev);
        spit_mat(d + "out_mapper.yuv", out);
        spit_mat(d + "out_preview.rgb", prev);
        {
            std::ofstream g(d + "gains_mapper.txt");
            g.precision(17);
            for (double v : mapper.gains()) g << v << "\n";
        }

        // ---- AsyncMultiMapper::New + push / pop (async.cpp:174-193) ---------------------------------
        std::vector<vr::MapperTemplate> mts{mt2};
        std::unique_ptr<vr::AsyncMultiMapper> am(vr::AsyncMultiMapper::New(
            mts, sizes, mt2.out_size, {blend}, {0}, {cv::Rect_<double>(0, 0, 1, 1)}, cv::Size(pw, ph)));
        const int frames_n = 3;
        std::vector<std::vector<std::tuple<cv::Mat, cv::Mat, cv::Mat>>> ins(frames_n);
        std::vector<std::tuple<cv::Mat, cv::Mat, cv::Mat>> outs(frames_n);
        for (int f = 0; f < frames_n; f++) {
            for (int i = 0; i < n; i++) {
                const int w = sizes[i].width, h = sizes[i].height;
                cv::Mat Y(h, w, CV_8UC1), U(h / 2, w / 2, CV_8UC1), V(h / 2, w / 2, CV_8UC1);
                for (int r = 0; r < h; r++)
                    for (int c = 0; c < w; c++) Y.at<uint8_t>(r, c) = (uint8_t)(frames[i].at<uint8_t>(r, c) + 11 * f);
                for (int r = 0; r < h / 2; r++)
                    for (int c = 0; c < w / 2; c++) {
                        U.at<uint8_t>(r, c) = frames[i].at<uint8_t>(h + r, c);
                        V.at<uint8_t>(r, c) = frames[i].at<uint8_t>(h + r, w / 2 + c);
                    }
                ins[f].emplace_back(Y, U, V);
            }
            outs[f] = std::make_tuple(cv::Mat(H, W, CV_8UC1), cv::Mat(H / 2, W / 2, CV_8UC1), cv::Mat(H / 2, W / 2, CV_8UC1));
            am->push(ins[f], outs[f]);
        }
        for (int f = 0; f < frames_n; f++) {
            am->pop();
            spit_mat(d + "out_async" + std::to_string(f) + "_y", std::get<0>(outs[f]));
            spit_mat(d + "out_async" + std::to_string(f) + "_u", std::get<1>(outs[f]));
            spit_mat(d + "out_async" + std::to_string(f) + "_v", std::get<2>(outs[f]));
        }
        {  // the preview of the last frame (async.cpp:149-171) and its PreviewDataHeader
            cv::Mat pv;
            vr::PreviewDataHeader hdr{};
            if (!am->preview(pv, hdr)) throw std::runtime_error("no preview published");
            spit_mat(d + "out_async_preview.rgb", pv);
            std::ofstream(d + "preview_hdr.txt") << hdr.width << " " << hdr.height << " " << hdr.step << "\n";
        }
        am.reset();

        // ---- FastMapper::stitch_nv12 on a template without ROI (octvr_dump -n; map.cpp:91-129) -------
        vr::MapperTemplate mt3(out_type, out_opts, W, H);
        for (int i = 0; i < n; i++) mt3.add_input(types[i], opts[i], false, false);
        vr::FastMapper fm(mt3, sizes);
        std::vector<cv::UMat> nv12(n);
        for (int i = 0; i < n; i++) {
            const int w = sizes[i].width, h = sizes[i].height;
            cv::Mat m(h * 3 / 2, w, CV_8UC1);
            for (int r = 0; r < h; r++) memcpy(m.ptr(r), frames[i].ptr(r), (size_t)w);
            for (int r = 0; r < h / 2; r++)
                for (int c = 0; c < w / 2; c++) {
                    m.at<uint8_t>(h + r, 2 * c) = frames[i].at<uint8_t>(h + r, c);               // U
                    m.at<uint8_t>(h + r, 2 * c + 1) = frames[i].at<uint8_t>(h + r, w / 2 + c);  // V
                }
            nv12[i] = cv::UMat(m);
        }
        cv::UMat fout;
        fm.stitch_nv12(nv12, fout);
        spit_mat(d + "out_fast.nv12", fout);
        bool threw = false;
        try {
            fm.stitch(nv12, fout);
        } catch (const cv::Exception&) {
            threw = true;  // mapper_fast.cpp:111-151
        }
        if (!threw) throw std::runtime_error("FastMapper::stitch should throw");

        // ---- errors as the reference raises them -----------------------------------------------------
        bool parse_err = false;
        try {
            std::ofstream bad(d + "bad.dat", std::ios::binary);
            bad << "VRv10 not a template";
            bad.close();
            std::ifstream bf(d + "bad.dat", std::ios::binary);
            vr::MapperTemplate broken(bf);
        } catch (const std::string& e) {  // template.cpp:262: throw std::string
            parse_err = e.find("version") != std::string::npos;
        }
        if (!parse_err) throw std::runtime_error("a bad .dat should throw std::string");
        vr::Timer t("api");
        t.tick("done");
        spit(d + "ok", "ok", 2);
        return 0;
    } catch (const std::string& e) {
        std::cerr << "error (std::string): " << e << std::endl;
    } catch (const std::exception& e) {
        std::cerr << "error: " << e.what() << std::endl;
    }
    return 1;
}
