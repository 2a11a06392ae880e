// Mutation fuzzing of the scene-file reader (csrc/rt_yaml.cpp) under
// AddressSanitizer + UndefinedBehaviorSanitizer (host code only):
//   g++ -std=c++17 -g -O1 -fsanitize=address,undefined -fno-sanitize-recover=all \
//       -Iraytracingthenextweekcuda_amd/csrc tools/yaml_fuzz.cpp \
//       raytracingthenextweekcuda_amd/csrc/rt_yaml.cpp -o /tmp/yaml_fuzz
//   /tmp/yaml_fuzz N_MUTATIONS file.yaml...
// Every mutant must either parse or return an error string; the sanitizers
// abort on any memory or UB fault. Prints the parse/error counts.
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>

#include "rt_yaml.h"

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint64_t next() {
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return rng_state;
}

static void walk(const rt::yaml::Node& n, int depth, long& count) {
    ++count;
    double d;
    long l;
    bool b;
    (void)rt::yaml::as_double(n, d);
    (void)rt::yaml::as_int(n, l);
    (void)rt::yaml::as_bool(n, b);
    for (const auto& kv : n.map) walk(kv.second, depth + 1, count);
    for (const auto& c : n.seq) walk(c, depth + 1, count);
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const long n = atol(argv[1]);
    const char alphabet[] = "-:#[]{}, \n\t01.e'\"&*|>!abc";
    long ok = 0, err = 0, nodes = 0;
    for (int f = 2; f < argc; ++f) {
        std::ifstream in(argv[f], std::ios::binary);
        std::stringstream ss;
        ss << in.rdbuf();
        const std::string base = ss.str();
        for (long i = 0; i < n; ++i) {
            std::string t = base;
            const int edits = 1 + (int)(next() % 4);
            for (int e = 0; e < edits && !t.empty(); ++e) {
                const size_t pos = next() % t.size();
                switch (next() % 4) {
                    case 0: t[pos] = alphabet[next() % (sizeof(alphabet) - 1)]; break;
                    case 1: t.insert(pos, 1, alphabet[next() % (sizeof(alphabet) - 1)]); break;
                    case 2: t.erase(pos, 1 + next() % 8); break;
                    default: t.resize(pos); break;
                }
            }
            rt::yaml::Node root;
            const std::string e = rt::yaml::parse(t, root);
            if (e.empty()) {
                ++ok;
                walk(root, 0, nodes);
            } else {
                ++err;
            }
        }
    }
    // hostile nesting: deep flow brackets and a staircase of indentation
    for (int k : {10, 1000, 100000}) {
        rt::yaml::Node root;
        std::string deep = "a: " + std::string((size_t)k, '[') + std::string((size_t)k, ']') + "\n";
        std::string stairs;
        for (int j = 0; j < k && j < 20000; ++j) stairs += std::string((size_t)j, ' ') + "k" + std::to_string(j) + ":\n";
        (rt::yaml::parse(deep, root).empty() ? ok : err)++;
        (rt::yaml::parse(stairs, root).empty() ? ok : err)++;
    }
    std::printf("mutants parsed %ld, rejected %ld, nodes walked %ld\n", ok, err, nodes);
    return 0;
}
