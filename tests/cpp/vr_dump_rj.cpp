// vr_dump_rj — the reference's template dumper flow (apps/octvr/dump.cpp:71-113) through the
// rapidjson::Value overloads of include/octvr.hpp (octvr.hpp:75-84 in the reference).  Built by build()
// only where rapidjson's headers exist (the reference vendors rapidjson 1.0.2 under
// modules/octvr/include; it is used from there at compile time, nothing is copied), and run by
// tests/test_gpu_cpp_api.py (the .dat against the reference's bytes) and tests/test_json_locale.py.
//
// Like the Qt application that embeds the reference, it calls setlocale(LC_ALL, "") first, so a
// comma-decimal LC_NUMERIC in the environment is active while the options travel through the API.
//
//   vr_dump_rj [-w W] [-h H] [-c] [-n] -o OUT.dat CONFIG.json   dump.cpp's flow
//   vr_dump_rj -s [-w W] [-h H] CONFIG.json                     template ctor only (no GPU): prints
//                                                              "W H" and printf's "%g" of 1.5
#include <unistd.h>

#include <clocale>
#include <cstdio>
#include <fstream>
#include <iostream>

#include "octvr.hpp"
#include "rapidjson/document.h"
#include "rapidjson/istreamwrapper.h"

#ifndef OCTVR_HAVE_RAPIDJSON
#error "vr_dump_rj needs the rapidjson::Value overloads of octvr.hpp"
#endif

using namespace vr;

int main(int argc, char* const argv[]) {
    std::setlocale(LC_ALL, "");  // as QApplication does
    int opt_width = 0, opt_height = 0;
    const char* opt_outfile = nullptr;
    bool opt_control_points = false, opt_roi = true, opt_size_only = false;
    int c;
    while ((c = getopt(argc, argv, "w:h:o:cns")) != -1) {
        switch (c) {
            case 'w': opt_width = atoi(optarg); break;
            case 'h': opt_height = atoi(optarg); break;
            case 'o': opt_outfile = optarg; break;
            case 'c': opt_control_points = true; break;
            case 'n': opt_roi = false; break;
            case 's': opt_size_only = true; break;
            default: return 2;
        }
    }
    if (optind >= argc || (!opt_outfile && !opt_size_only)) {
        fprintf(stderr, "usage: %s [-w W] [-h H] [-c] [-n] (-o OUT | -s) CONFIG\n", argv[0]);
        return 2;
    }
    try {
        rapidjson::Document options;
        std::ifstream f(argv[optind]);
        rapidjson::IStreamWrapper ifs(f);
        options.ParseStream(ifs);
        if (options.HasParseError()) throw std::string("bad config json");

        MapperTemplate mt(options["output"]["type"].GetString(), options["output"]["options"], opt_width, opt_height);
        if (opt_size_only) {
            printf("%d %d %g\n", mt.out_size.width, mt.out_size.height, 1.5);
            return 0;
        }
        for (auto i = options["inputs"].Begin(); i != options["inputs"].End(); i++)
            mt.add_input((*i)["type"].GetString(), (*i)["options"], false, opt_roi);
        if (options.HasMember("overlays"))
            for (auto i = options["overlays"].Begin(); i != options["overlays"].End(); i++)
                mt.add_input((*i)["type"].GetString(), (*i)["options"], true, opt_roi);
        if (opt_control_points && options.HasMember("control_points")) mt.morph_controlpoints(options["control_points"]);
        std::ofstream of(opt_outfile, std::ios::binary);
        mt.dump(of);
        fprintf(stderr, "dumped %d inputs, %dx%d\n", (int)mt.inputs.size(), mt.out_size.width, mt.out_size.height);
        return 0;
    } catch (const std::string& e) {
        std::cerr << "error (std::string): " << e << std::endl;
    } catch (const std::exception& e) {
        std::cerr << "error: " << e.what() << std::endl;
    }
    return 1;
}
