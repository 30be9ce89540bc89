// xml.cpp — see xml.h.  A small DOM reader (no pugixml in this image) plus the
// reference's DFS visitor semantics (resource/xml/visitor.h:98-194).
#include "xml.h"

#include <algorithm>
#include <cctype>
#include <fstream>
#include <sstream>

namespace Pupil::resource::xml {

std::string Object::GetProperty(std::string_view name) const {
    for (auto &p : properties)
        if (p.name == name) return p.value;
    return "";
}

Object *Object::GetUniqueSubObject(std::string_view name) const {
    for (auto *so : sub_object)
        if (so->obj_name == name) return so;
    return nullptr;
}

std::vector<Object *> Object::GetSubObjects(std::string_view name) const {
    std::vector<Object *> ret;
    for (auto *so : sub_object)
        if (so->obj_name == name) ret.push_back(so);
    return ret;
}

std::pair<Object *, std::string> Object::GetParameter(std::string_view name) const {
    for (auto *so : sub_object)
        if (so->var_name == name) return {so, ""};
    return {nullptr, GetProperty(name)};
}

namespace {

struct Node {
    std::string name;
    std::vector<std::pair<std::string, std::string>> attrs;
    std::vector<std::unique_ptr<Node>> children;

    bool has(const std::string &k) const {
        for (auto &a : attrs)
            if (a.first == k) return true;
        return false;
    }
    std::string get(const std::string &k) const {
        for (auto &a : attrs)
            if (a.first == k) return a.second;
        return "";
    }
    void set(const std::string &k, const std::string &v) {
        for (auto &a : attrs)
            if (a.first == k) a.second = v;
    }
};

class Reader {
public:
    explicit Reader(const std::string &t) : s(t) {}
    std::unique_ptr<Node> parse_document(std::string &err) {
        std::unique_ptr<Node> root;
        while (true) {
            skip_misc();
            if (i >= s.size()) break;
            if (s[i] != '<') {
                err = "unexpected text outside the root element";
                return nullptr;
            }
            auto n = parse_element(err);
            if (!n) return nullptr;
            if (!root) root = std::move(n);
        }
        if (!root) err = "empty document";
        return root;
    }

private:
    const std::string &s;
    size_t i = 0;

    void skip_ws() {
        while (i < s.size() && std::isspace((unsigned char)s[i])) i++;
    }
    // whitespace, comments, processing instructions, doctype
    void skip_misc() {
        while (true) {
            skip_ws();
            if (s.compare(i, 4, "<!--") == 0) {
                size_t e = s.find("-->", i + 4);
                i = e == std::string::npos ? s.size() : e + 3;
            } else if (s.compare(i, 2, "<?") == 0) {
                size_t e = s.find("?>", i + 2);
                i = e == std::string::npos ? s.size() : e + 2;
            } else if (s.compare(i, 2, "<!") == 0) {
                size_t e = s.find('>', i + 2);
                i = e == std::string::npos ? s.size() : e + 1;
            } else {
                return;
            }
        }
    }
    static std::string unescape(const std::string &v) {
        std::string out;
        for (size_t k = 0; k < v.size(); k++) {
            if (v[k] == '&') {
                const size_t e = v.find(';', k);
                if (e != std::string::npos) {
                    const std::string ent = v.substr(k + 1, e - k - 1);
                    if (ent == "lt") out += '<';
                    else if (ent == "gt") out += '>';
                    else if (ent == "amp") out += '&';
                    else if (ent == "quot") out += '"';
                    else if (ent == "apos") out += '\'';
                    else out += v.substr(k, e - k + 1);
                    k = e;
                    continue;
                }
            }
            out += v[k];
        }
        return out;
    }
    std::string parse_name() {
        size_t b = i;
        while (i < s.size() && (std::isalnum((unsigned char)s[i]) || s[i] == '_' || s[i] == '-' || s[i] == ':' ||
                                s[i] == '.'))
            i++;
        return s.substr(b, i - b);
    }
    std::unique_ptr<Node> parse_element(std::string &err) {
        auto n = std::make_unique<Node>();
        i++;  // '<'
        n->name = parse_name();
        if (n->name.empty()) {
            err = "malformed element";
            return nullptr;
        }
        while (true) {
            skip_ws();
            if (i >= s.size()) {
                err = "unterminated element <" + n->name + ">";
                return nullptr;
            }
            if (s[i] == '/') {
                if (s.compare(i, 2, "/>") != 0) {
                    err = "malformed empty element";
                    return nullptr;
                }
                i += 2;
                return n;
            }
            if (s[i] == '>') {
                i++;
                break;
            }
            std::string key = parse_name();
            skip_ws();
            if (key.empty() || i >= s.size() || s[i] != '=') {
                err = "malformed attribute in <" + n->name + ">";
                return nullptr;
            }
            i++;
            skip_ws();
            if (i >= s.size() || (s[i] != '"' && s[i] != '\'')) {
                err = "unquoted attribute value";
                return nullptr;
            }
            const char q = s[i++];
            const size_t e = s.find(q, i);
            if (e == std::string::npos) {
                err = "unterminated attribute value";
                return nullptr;
            }
            n->attrs.emplace_back(key, unescape(s.substr(i, e - i)));
            i = e + 1;
        }
        // children
        while (true) {
            // text content is ignored (the reference reads attributes only)
            while (i < s.size() && s[i] != '<') i++;
            if (i >= s.size()) {
                err = "missing </" + n->name + ">";
                return nullptr;
            }
            if (s.compare(i, 4, "<!--") == 0 || s.compare(i, 2, "<?") == 0 ||
                (s.compare(i, 2, "<!") == 0)) {
                skip_misc();
                continue;
            }
            if (s.compare(i, 2, "</") == 0) {
                i += 2;
                const std::string close = parse_name();
                skip_ws();
                if (close != n->name || i >= s.size() || s[i] != '>') {
                    err = "mismatched </" + close + "> for <" + n->name + ">";
                    return nullptr;
                }
                i++;
                return n;
            }
            auto c = parse_element(err);
            if (!c) return nullptr;
            n->children.push_back(std::move(c));
        }
    }
};

enum class Tag {
    unknown, scene, default_, bsdf, emitter, film, integrator, sensor, shape, texture, lookat, transform,
    integer, string, float_, rgb, point, matrix, scale, rotate, translate, boolean, ref
};

Tag tag_of(const std::string &n) {
    static const std::unordered_map<std::string, Tag> m = {
        {"scene", Tag::scene},     {"default", Tag::default_},     {"bsdf", Tag::bsdf},
        {"emitter", Tag::emitter}, {"film", Tag::film},            {"integrator", Tag::integrator},
        {"sensor", Tag::sensor},   {"shape", Tag::shape},          {"texture", Tag::texture},
        {"lookat", Tag::lookat},   {"transform", Tag::transform},  {"integer", Tag::integer},
        {"string", Tag::string},   {"float", Tag::float_},         {"rgb", Tag::rgb},
        {"point", Tag::point},     {"matrix", Tag::matrix},        {"scale", Tag::scale},
        {"rotate", Tag::rotate},   {"translate", Tag::translate},  {"boolean", Tag::boolean},
        {"ref", Tag::ref}};
    auto it = m.find(n);
    return it == m.end() ? Tag::unknown : it->second;
}

struct Visitor {
    std::vector<std::unique_ptr<Object>> &pool;
    Object *current = nullptr;
    Object *root = nullptr;
    std::map<std::string, std::string> params;
    std::unordered_map<std::string, Object *> refs;

    // GlobalManager::ReplaceDefaultValue (object.cpp:9-24); longest names first
    void replace_defaults(Node &n) {
        std::vector<std::pair<std::string, std::string>> ps(params.begin(), params.end());
        std::sort(ps.begin(), ps.end(), [](auto &a, auto &b) { return a.first.size() > b.first.size(); });
        for (auto &a : n.attrs) {
            if (a.second.find('$') == std::string::npos) continue;
            for (auto &[name, value] : ps) {
                const std::string key = "$" + name;
                size_t pos = 0;
                while ((pos = a.second.find(key, pos)) != std::string::npos) {
                    a.second.replace(pos, key.size(), value);
                    pos += value.size();
                }
            }
        }
    }
    Object *new_object(const std::string &name, const std::string &type) {
        pool.push_back(std::make_unique<Object>());
        Object *o = pool.back().get();
        o->obj_name = name;
        o->type = type;
        return o;
    }
    void add_property(const std::string &name, const std::string &value) {
        if (current) current->properties.push_back({name, value});
    }
    bool xyz_property(Node &n, const char *dx, const char *dy, const char *dz) {
        replace_defaults(n);
        std::string name = n.get("name");
        if (name.empty()) name = n.name;
        std::string value = n.get("value");
        if (value.empty()) {
            std::string x = n.get("x"), y = n.get("y"), z = n.get("z");
            if (x.empty()) x = dx;
            if (y.empty()) y = dy;
            if (z.empty()) z = dz;
            value = x + "," + y + "," + z;
        }
        add_property(name, value);
        return true;
    }
    bool visit(Node &n) {
        switch (tag_of(n.name)) {
            case Tag::scene: {
                Object *o = new_object(n.name, n.get("version"));
                current = o;
                if (!root) root = o;
                return true;
            }
            case Tag::default_:
                replace_defaults(n);
                params[n.get("name")] = n.get("value");
                return true;
            case Tag::ref: {
                replace_defaults(n);
                auto it = refs.find(n.get("id"));
                if (it != refs.end() && current) current->sub_object.push_back(it->second);
                return true;
            }
            case Tag::lookat: {
                replace_defaults(n);
                Object *o = new_object(n.name, "");
                for (const char *k : {"origin", "target", "up"})
                    if (n.has(k)) o->properties.push_back({k, n.get(k)});
                if (current) current->sub_object.push_back(o);
                return true;
            }
            case Tag::rotate: {
                replace_defaults(n);
                Object *o = new_object(n.name, "");
                std::string axis;
                if (n.has("value")) axis = n.get("value");
                else if (n.has("x")) axis = "1, 0, 0";
                else if (n.has("y")) axis = "0, 1, 0";
                else if (n.has("z")) axis = "0, 0, 1";
                o->properties.push_back({"axis", axis});
                o->properties.push_back({"angle", n.get("angle")});
                if (current) current->sub_object.push_back(o);
                return true;
            }
            case Tag::scale: return xyz_property(n, "1", "1", "1");
            case Tag::point:
            case Tag::translate: return xyz_property(n, "0", "0", "0");
            case Tag::integer:
            case Tag::string:
            case Tag::float_:
            case Tag::rgb:
            case Tag::boolean:
            case Tag::matrix: {
                replace_defaults(n);
                std::string name = n.get("name");
                if (name.empty()) name = n.name;
                add_property(name, n.get("value"));
                return true;
            }
            case Tag::bsdf:
            case Tag::emitter:
            case Tag::film:
            case Tag::integrator:
            case Tag::sensor:
            case Tag::shape:
            case Tag::texture:
            case Tag::transform: {
                replace_defaults(n);
                Object *o = new_object(n.name, n.get("type"));
                if (n.has("id")) {
                    o->id = n.get("id");
                    refs[o->id] = o;
                }
                if (n.has("name")) o->var_name = n.get("name");
                if (current) current->sub_object.push_back(o);
                current = o;
                return true;
            }
            default: return false;  // unknown tags (sampler, rfilter, ...) are skipped with their subtree
        }
    }
    void dfs(Node &n) {
        Object *parent = current;
        if (!visit(n)) return;
        for (auto &c : n.children) dfs(*c);
        current = parent;
    }
};

}  // namespace

Object *Parser::LoadFromString(const std::string &text, std::string *error) {
    std::string err;
    Reader r(text);
    auto root = r.parse_document(err);
    if (!root) {
        if (error) *error = err;
        return nullptr;
    }
    Visitor v{m_pool};
    v.dfs(*root);
    if (!v.root) {
        if (error) *error = "document root is not <scene>";
        return nullptr;
    }
    return v.root;
}

Object *Parser::LoadFromFile(const std::string &path, std::string *error) {
    std::ifstream f(path, std::ios::binary);
    if (!f) {
        if (error) *error = "cannot open " + path;
        return nullptr;
    }
    std::stringstream ss;
    ss << f.rdbuf();
    return LoadFromString(ss.str(), error);
}

}  // namespace Pupil::resource::xml
