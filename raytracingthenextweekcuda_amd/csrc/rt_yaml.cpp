// Minimal block-style YAML reader (see rt_yaml.h).
#include "rt_yaml.h"

#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

namespace rt {
namespace yaml {

const Node* Node::get(const std::string& key) const {
    if (kind != kMap) return nullptr;
    for (const auto& kv : map)
        if (kv.first == key) return &kv.second;
    return nullptr;
}

namespace {

struct Line {
    int indent;
    std::string text;  // without indentation, comment and trailing blanks
    int number;
};

std::string trim(const std::string& s) {
    size_t b = 0, e = s.size();
    while (b < e && (s[b] == ' ' || s[b] == '\t')) ++b;
    while (e > b && (s[e - 1] == ' ' || s[e - 1] == '\t' || s[e - 1] == '\r')) --e;
    return s.substr(b, e - b);
}

std::string err_at(int line, const std::string& msg) { return "line " + std::to_string(line) + ": " + msg; }

// A `#` starts a comment at the start of the content or after a blank; quoted
// scalars are not used by the scene files, so quotes are not tracked.
std::string strip_comment(const std::string& s) {
    for (size_t i = 0; i < s.size(); ++i)
        if (s[i] == '#' && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '\t')) return s.substr(0, i);
    return s;
}

// "key: value" / "key:" -> true with key and value (value may be empty).
bool split_key(const std::string& t, std::string& key, std::string& value) {
    for (size_t i = 0; i < t.size(); ++i) {
        if (t[i] == ':' && (i + 1 == t.size() || t[i + 1] == ' ')) {
            key = trim(t.substr(0, i));
            value = trim(t.substr(i + 1));
            return !key.empty();
        }
    }
    return false;
}

class Parser {
public:
    explicit Parser(std::vector<Line> lines) : L(std::move(lines)) {}

    std::string document(Node& root) {
        if (L.empty()) {
            root = Node{};
            return "";
        }
        std::string e = block(0, L[0].indent, root);
        if (!e.empty()) return e;
        if (i < L.size()) return err_at(L[i].number, "unexpected indentation");
        return "";
    }

private:
    std::vector<Line> L;
    size_t i = 0;
    int depth = 0;  // nesting guard: scene files nest 4 levels; hostile input must not exhaust the stack
    static constexpr int kMaxDepth = 128;

    struct Nest {
        int& d;
        explicit Nest(int& x) : d(x) { ++d; }
        ~Nest() { --d; }
    };

    static bool is_item(const std::string& t) { return t == "-" || (t.size() > 1 && t[0] == '-' && t[1] == ' '); }

    // Flow collections ([a, b], {k: v}, nested) and plain scalars.
    static void skip_ws(const std::string& v, size_t& p) {
        while (p < v.size() && v[p] == ' ') ++p;
    }

    std::string flow(const std::string& v, size_t& p, int line, Node& out) {
        Nest guard(depth);
        if (depth > kMaxDepth) return err_at(line, "nesting too deep");
        skip_ws(v, p);
        out = Node{};
        out.line = line;
        if (p >= v.size()) return err_at(line, "unterminated flow collection");
        const char open = v[p];
        if (open == '[' || open == '{') {
            const char close = open == '[' ? ']' : '}';
            out.kind = open == '[' ? Node::kSeq : Node::kMap;
            ++p;
            skip_ws(v, p);
            if (p < v.size() && v[p] == close) {
                ++p;
                return "";
            }
            for (;;) {
                std::string key;
                if (open == '{') {
                    const size_t colon = v.find(':', p);
                    if (colon == std::string::npos) return err_at(line, "expected 'key: value' in flow map");
                    key = trim(v.substr(p, colon - p));
                    if (key.empty()) return err_at(line, "empty key in flow map");
                    p = colon + 1;
                }
                Node item;
                std::string e = flow(v, p, line, item);
                if (!e.empty()) return e;
                if (open == '{') out.map.emplace_back(key, std::move(item));
                else out.seq.push_back(std::move(item));
                skip_ws(v, p);
                if (p < v.size() && v[p] == ',') {
                    ++p;
                    continue;
                }
                if (p < v.size() && v[p] == close) {
                    ++p;
                    return "";
                }
                return err_at(line, "unterminated flow collection");
            }
        }
        // plain scalar up to the next delimiter of the enclosing flow collection
        size_t q = p;
        while (q < v.size() && v[q] != ',' && v[q] != ']' && v[q] != '}') ++q;
        out.kind = Node::kScalar;
        out.scalar = trim(v.substr(p, q - p));
        p = q;
        if (out.scalar.empty()) return err_at(line, "empty flow item");
        return "";
    }

    std::string scalar(const std::string& v, int line, Node& out) {
        out = Node{};
        out.line = line;
        if (v.empty()) return "";  // null
        if (v[0] == '&' || v[0] == '*' || v[0] == '|' || v[0] == '>' || v[0] == '!')
            return err_at(line, "unsupported YAML construct '" + v.substr(0, 1) + "'");
        if (v[0] == '[' || v[0] == '{') {
            size_t p = 0;
            std::string e = flow(v, p, line, out);
            if (!e.empty()) return e;
            skip_ws(v, p);
            if (p != v.size()) return err_at(line, "trailing characters after flow collection");
            return "";
        }
        std::string s = v;
        if (s.size() >= 2 && ((s.front() == '"' && s.back() == '"') || (s.front() == '\'' && s.back() == '\'')))
            s = s.substr(1, s.size() - 2);
        out.kind = Node::kScalar;
        out.scalar = s;
        return "";
    }

    // The value block of a `key:` or `-` with nothing after it: the following
    // lines indented deeper than `parent`, or a sequence at the same indent
    // (YAML allows `key:` followed by `- item` at the key's column).
    std::string child(int parent, bool allow_same_indent_seq, int line, Node& out) {
        if (i < L.size() && (L[i].indent > parent || (allow_same_indent_seq && L[i].indent == parent &&
                                                       is_item(L[i].text))))
            return block(i, L[i].indent, out);
        out = Node{};
        out.line = line;
        return "";
    }

    std::string block(size_t start, int indent, Node& out) {
        Nest guard(depth);
        if (depth > kMaxDepth) return err_at(L[start].number, "nesting too deep");
        i = start;
        out = Node{};
        out.line = L[i].number;
        if (is_item(L[i].text)) return sequence(indent, out);
        return mapping(indent, out);
    }

    std::string sequence(int indent, Node& out) {
        out.kind = Node::kSeq;
        while (i < L.size() && L[i].indent == indent && is_item(L[i].text)) {
            const Line ln = L[i];
            const std::string rest = trim(ln.text.substr(1));
            Node item;
            if (rest.empty()) {
                ++i;
                std::string e = child(indent, false, ln.number, item);
                if (!e.empty()) return e;
            } else {
                std::string k, v;
                if (rest[0] != '[' && rest[0] != '{' && split_key(rest, k, v)) {
                    // "- key: ..." opens a map whose first entry sits on this line
                    const int col = indent + (int)ln.text.find_first_not_of(' ', 1);
                    L[i].indent = col;
                    L[i].text = rest;
                    std::string e = block(i, col, item);
                    if (!e.empty()) return e;
                } else {
                    std::string e = scalar(rest, ln.number, item);
                    if (!e.empty()) return e;
                    ++i;
                }
            }
            out.seq.push_back(std::move(item));
        }
        if (i < L.size() && L[i].indent > indent) return err_at(L[i].number, "unexpected indentation");
        return "";
    }

    std::string mapping(int indent, Node& out) {
        out.kind = Node::kMap;
        while (i < L.size() && L[i].indent == indent && !is_item(L[i].text)) {
            const Line ln = L[i];
            std::string k, v;
            if (!split_key(ln.text, k, v)) return err_at(ln.number, "expected 'key: value'");
            for (const auto& kv : out.map)
                if (kv.first == k) return err_at(ln.number, "duplicate key '" + k + "'");
            ++i;
            Node val;
            std::string e = v.empty() ? child(indent, true, ln.number, val) : scalar(v, ln.number, val);
            if (!e.empty()) return e;
            out.map.emplace_back(k, std::move(val));
        }
        if (i < L.size() && L[i].indent > indent) return err_at(L[i].number, "unexpected indentation");
        return "";
    }
};

}  // namespace

std::string parse(const std::string& text, Node& root) {
    std::vector<Line> lines;
    std::stringstream ss(text);
    std::string raw;
    int number = 0;
    while (std::getline(ss, raw)) {
        ++number;
        std::string s = strip_comment(raw);
        size_t ind = 0;
        while (ind < s.size() && s[ind] == ' ') ++ind;
        if (ind < s.size() && s[ind] == '\t') return err_at(number, "tab indentation");
        std::string t = trim(s);
        if (t.empty()) continue;
        if (t == "---" && lines.empty()) continue;
        if (t == "---" || t == "...") return err_at(number, "multi-document streams are not supported");
        lines.push_back({(int)ind, t, number});
    }
    Parser p(std::move(lines));
    return p.document(root);
}

std::string parse_file(const std::string& path, Node& root) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return "cannot open " + path;
    std::stringstream buf;
    buf << f.rdbuf();
    return parse(buf.str(), root);
}

bool as_double(const Node& n, double& out) {
    if (n.kind != Node::kScalar || n.scalar.empty()) return false;
    const char* s = n.scalar.c_str();
    char* end = nullptr;
    errno = 0;
    const double v = std::strtod(s, &end);
    if (end == s || *end != '\0' || errno == ERANGE) return false;
    // strtod also takes "inf", "nan" and hex floats; YAML spells those differently
    for (const char* p = s; *p; ++p)
        if (!std::strchr("+-.0123456789eE", *p)) return false;
    out = v;
    return true;
}

bool as_int(const Node& n, long& out) {
    if (n.kind != Node::kScalar || n.scalar.empty()) return false;
    const char* s = n.scalar.c_str();
    char* end = nullptr;
    errno = 0;
    const long v = std::strtol(s, &end, 10);
    if (end == s || *end != '\0' || errno == ERANGE) return false;
    out = v;
    return true;
}

bool as_bool(const Node& n, bool& out) {
    if (n.kind != Node::kScalar) return false;
    const std::string& s = n.scalar;
    // YAML 1.1 booleans, as PyYAML resolves them
    if (s == "true" || s == "True" || s == "TRUE" || s == "yes" || s == "Yes" || s == "YES" || s == "on" ||
        s == "On" || s == "ON") {
        out = true;
        return true;
    }
    if (s == "false" || s == "False" || s == "FALSE" || s == "no" || s == "No" || s == "NO" || s == "off" ||
        s == "Off" || s == "OFF") {
        out = false;
        return true;
    }
    return false;
}

}  // namespace yaml
}  // namespace rt
