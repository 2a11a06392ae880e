// Minimal YAML reader for the reference's scene files (resources/scenes), which
// the reference reads with yaml-cpp 0.7.0 (main.cu:623-786; the library binary
// is not in the reference tree). It covers what those files and their re-dumps
// use: block maps, `- item` sequences (scalars or maps, including the
// `- plane:` first-key form), `# comments`, a leading `---`, and one-line flow
// collections (`[0, 1, 0]`, `{type: 0, albedo: [1, 1, 1]}`). Anchors, tags,
// block scalars and multi-document streams are rejected with the line number.
#pragma once

#include <string>
#include <utility>
#include <vector>

namespace rt {
namespace yaml {

struct Node {
    enum Kind { kNull, kScalar, kMap, kSeq } kind = kNull;
    std::string scalar;
    std::vector<std::pair<std::string, Node>> map;  // document order kept (first-key rule)
    std::vector<Node> seq;
    int line = 0;  // 1-based source line

    const Node* get(const std::string& key) const;
};

// Parses `text`; returns "" on success or "line N: message".
std::string parse(const std::string& text, Node& root);
std::string parse_file(const std::string& path, Node& root);

// Scalar conversions with YAML 1.1 core rules as PyYAML applies them to these
// files: ints, floats (strtod on the whole token) and true/false. Each returns
// false when the node is not a scalar of that type.
bool as_double(const Node& n, double& out);
bool as_int(const Node& n, long& out);
bool as_bool(const Node& n, bool& out);

}  // namespace yaml
}  // namespace rt
