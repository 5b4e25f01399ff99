// quant -- command-line front end of the MI355X codec, with the reference's flags and defaults
// (src/main.cpp:42-113, no Boost):
//
//   quant FILE -o OUT [-n bits=8] [-e eps=1e-6] [-w width=2] [-h height=2] [-r raport=0]
//                     [-q quantizer=0 (LBG)] [-c colorspace=1 (SCALED)] [--device N]
//
// FILE.ppm -> OUT.quant compresses, FILE.quant -> OUT.ppm decompresses, FILE.ppm -> OUT.ppm
// compresses and writes the decoded image (src/main.cpp:73-111); anything else prints "File
// type not supported" and exits 1.  Options take a value as "-n 8", "-n8", "--saveto OUT" or
// "--saveto=OUT" (program_options' short and long forms); -r takes a value ("-r 1"), -h is the
// block height and --help the help text, as in the reference.  The quantization itself runs
// on the GPU through libquant_amd.so / libqvq.so.
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <map>
#include <stdexcept>
#include <string>

#include "quant_amd/Compressor.hpp"

namespace {

enum class FileType { NOT_SUPPORTED, PPM, QUANT };

// src/main.cpp:20-40: the extension after the last '.', unless a '/' comes first
FileType file_type(const std::string &path) {
    for (size_t i = path.size(); i-- > 0;) {
        if (path[i] == '/') return FileType::NOT_SUPPORTED;
        if (path[i] == '.') {
            const std::string ext = path.substr(i);
            if (ext == ".quant") return FileType::QUANT;
            if (ext == ".ppm") return FileType::PPM;
            return FileType::NOT_SUPPORTED;
        }
    }
    return FileType::NOT_SUPPORTED;
}

struct Params {   // include/ProgramParameters.hpp:5-19, defaults of src/main.cpp:49-57
    int n = 8, width = 2, height = 2, quantizer = (int)Quantizers::LBG, colorspace = (int)ColorSpaces::SCALED;
    float eps = 0.000001f;
    bool raport = false;
    std::string file, saveto;
};

const char *kHelp =
    "Options:\n"
    "  --help                 Print help messages\n"
    "  -n arg (=8)            bits per codevector\n"
    "  -e arg (=9.99999997e-07) eps parameter for quantization algorithm\n"
    "  -w arg (=2)            Width of block\n"
    "  -h arg (=2)            Height of block\n"
    "  --file arg             File to compress/decompress\n"
    "  -o [ --saveto ] arg    Save to\n"
    "  -r arg (=0)            Print raport to std::out\n"
    "  -q [ --quantizer ] arg (=0) Pick quantizer\n"
    "  -c [ --colorspace ] arg (=1) Pick ColorSpace\n"
    "  --device arg (=0)      HIP device of the engine (MI355X build)\n";

bool parse_bool(const std::string &v) {   // program_options' bool values
    if (v == "1" || v == "true" || v == "yes" || v == "on") return true;
    if (v == "0" || v == "false" || v == "no" || v == "off") return false;
    throw std::invalid_argument("the argument ('" + v + "') for option '-r' is invalid");
}

int parse_int(const std::string &v, const std::string &opt) {
    size_t pos = 0;
    const int x = std::stoi(v, &pos);
    if (pos != v.size()) throw std::invalid_argument("the argument ('" + v + "') for option '" + opt + "' is invalid");
    return x;
}

// Returns true when --help was given.
bool parse(int argc, char **argv, Params &p) {
    // option name -> canonical key; every option but --help takes a value
    const std::map<std::string, std::string> names = {
        {"-n", "n"}, {"-e", "e"}, {"-w", "w"}, {"-h", "h"}, {"-o", "o"}, {"--saveto", "o"}, {"-r", "r"},
        {"-q", "q"}, {"--quantizer", "q"}, {"-c", "c"}, {"--colorspace", "c"}, {"--c", "c"}, {"--file", "file"},
        {"--device", "device"}};
    bool have_file = false, have_out = false;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        if (a == "--help") return true;
        std::string key, val;
        bool has_val = false;
        if (a.size() > 1 && a[0] == '-') {
            std::string name = a;
            if (a.rfind("--", 0) == 0) {
                const size_t eq = a.find('=');
                if (eq != std::string::npos) {
                    name = a.substr(0, eq);
                    val = a.substr(eq + 1);
                    has_val = true;
                }
            } else if (a.size() > 2) {   // -n8
                name = a.substr(0, 2);
                val = a.substr(2);
                has_val = true;
            }
            const auto it = names.find(name);
            if (it == names.end()) throw std::invalid_argument("unrecognised option '" + a + "'");
            key = it->second;
            if (!has_val) {
                if (i + 1 >= argc) throw std::invalid_argument("the required argument for option '" + name + "' is missing");
                val = argv[++i];
            }
        } else {
            key = "file";   // positional
            val = a;
        }
        if (key == "n") p.n = parse_int(val, "-n");
        else if (key == "e") p.eps = std::stof(val);
        else if (key == "w") p.width = parse_int(val, "-w");
        else if (key == "h") p.height = parse_int(val, "-h");
        else if (key == "r") p.raport = parse_bool(val);
        else if (key == "q") p.quantizer = parse_int(val, "--quantizer");
        else if (key == "c") p.colorspace = parse_int(val, "--colorspace");
        else if (key == "device") setenv("QVQ_DEVICE", val.c_str(), 1);
        else if (key == "o") {
            p.saveto = val;
            have_out = true;
        } else {
            if (have_file) throw std::invalid_argument("option '--file' cannot be specified more than once");
            p.file = val;
            have_file = true;
        }
    }
    if (!have_file) throw std::invalid_argument("the option '--file' is required but missing");
    if (!have_out) throw std::invalid_argument("the option '--saveto' is required but missing");
    return false;
}

}  // namespace

int main(int argc, char **argv) {
    Params par;
    try {
        if (parse(argc, argv, par)) {
            std::cout << kHelp << std::endl;
            return 0;
        }
    } catch (const std::exception &e) {
        std::cerr << "quant: " << e.what() << std::endl;
        return 2;
    }
    const FileType from = file_type(par.file), to = file_type(par.saveto);
    try {
        auto run_compression = [&]() {   // src/main.cpp:76-84
            RGBImage img(par.file);
            auto result = CompressedImage::compress(img, (Quantizers)par.quantizer, (ColorSpaces)par.colorspace,
                                                    par.width, par.height, par.eps, par.n);
            if (par.raport) std::cout << result.second;
            return result.first;
        };
        auto run_decompression = [&](const CompressedImage &c) {   // src/main.cpp:86-90
            RGBImage out = CompressedImage::decompress(c);
            out.saveToFile(par.saveto);
        };
        if (from == FileType::PPM && to == FileType::PPM) {
            run_decompression(run_compression());
        } else if (from == FileType::QUANT && to == FileType::PPM) {
            CompressedImage c;
            c.loadFromFile(par.file);
            run_decompression(c);
        } else if (from == FileType::PPM && to == FileType::QUANT) {
            CompressedImage c = run_compression();
            c.saveToFile(par.saveto);
        } else {
            std::cerr << "File type not supported" << std::endl;
            return 1;
        }
    } catch (const std::exception &e) {
        std::cerr << "quant: " << e.what() << std::endl;
        return 3;
    }
    return 0;
}
