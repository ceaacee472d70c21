// xml.hpp — the small XML DOM the scene parser needs (what the reference gets from its
// vendored tinyxml2 4.0.1: elements, attributes in document order, the first text child of an
// element).  Comments, the <?xml?> declaration, <!DOCTYPE>, CDATA and the five predefined
// entities plus numeric character references are handled; namespaces are not.
#pragma once
#include <cstring>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace rtgh {

struct XmlElement {
    std::string name;
    std::vector<std::pair<std::string, std::string>> attrs;   // document order
    std::vector<std::unique_ptr<XmlElement>> children;
    std::string text;          // text before the first child element (tinyxml2 GetText())
    bool has_text = false;

    const XmlElement* child(const char* tag) const {          // FirstChildElement(tag)
        for (const auto& c : children)
            if (c->name == tag) return c.get();
        return nullptr;
    }
    std::vector<const XmlElement*> all(const char* tag) const {
        std::vector<const XmlElement*> v;
        for (const auto& c : children)
            if (c->name == tag) v.push_back(c.get());
        return v;
    }
    const std::string* attr(const char* key) const {
        for (const auto& a : attrs)
            if (a.first == key) return &a.second;
        return nullptr;
    }
};

class XmlParser {
public:
    // Returns the root element or nullptr (err set).
    std::unique_ptr<XmlElement> parse(const std::string& src, std::string& err) {
        s_ = src.data();
        n_ = src.size();
        p_ = 0;
        std::unique_ptr<XmlElement> root;
        while (true) {
            skip_ws();
            if (p_ >= n_) break;
            if (starts("<?")) { if (!skip_past("?>")) return fail(err, "unterminated declaration"); continue; }
            if (starts("<!--")) { if (!skip_past("-->")) return fail(err, "unterminated comment"); continue; }
            if (starts("<!")) { if (!skip_past(">")) return fail(err, "unterminated <!"); continue; }
            if (s_[p_] != '<') return fail(err, "text outside the root element");
            if (root) return fail(err, "more than one root element");
            root = element(err);
            if (!root) return nullptr;
        }
        if (!root) return fail(err, "no root element");
        return root;
    }

private:
    const char* s_ = nullptr;
    size_t n_ = 0, p_ = 0;

    std::unique_ptr<XmlElement> fail(std::string& err, const char* msg) {
        err = std::string("XML: ") + msg + " at byte " + std::to_string(p_);
        return nullptr;
    }
    bool starts(const char* t) const { size_t k = strlen(t); return p_ + k <= n_ && memcmp(s_ + p_, t, k) == 0; }
    bool skip_past(const char* t) {
        size_t k = strlen(t);
        while (p_ + k <= n_) {
            if (memcmp(s_ + p_, t, k) == 0) { p_ += k; return true; }
            p_++;
        }
        p_ = n_;
        return false;
    }
    void skip_ws() { while (p_ < n_ && (s_[p_] == ' ' || s_[p_] == '\t' || s_[p_] == '\n' || s_[p_] == '\r')) p_++; }
    static bool name_char(char c) {
        return !(c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '>' || c == '/' || c == '=' || c == '<' ||
                 c == '"' || c == '\'');
    }
    std::string name() {
        size_t b = p_;
        while (p_ < n_ && name_char(s_[p_])) p_++;
        return std::string(s_ + b, p_ - b);
    }
    static void put_utf8(std::string& o, unsigned cp) {
        if (cp < 0x80) o += (char)cp;
        else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); }
        else if (cp < 0x10000) { o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F)); }
        else { o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3F)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F)); }
    }
    static std::string unescape(const char* b, size_t len) {
        std::string o;
        o.reserve(len);
        for (size_t i = 0; i < len; i++) {
            if (b[i] != '&') { o += b[i]; continue; }
            size_t j = i + 1;
            while (j < len && b[j] != ';' && j - i < 12) j++;
            if (j >= len || b[j] != ';') { o += b[i]; continue; }
            std::string e(b + i + 1, j - i - 1);
            if (e == "lt") o += '<';
            else if (e == "gt") o += '>';
            else if (e == "amp") o += '&';
            else if (e == "quot") o += '"';
            else if (e == "apos") o += '\'';
            else if (!e.empty() && e[0] == '#') put_utf8(o, (unsigned)strtoul(e.c_str() + (e.size() > 1 && e[1] == 'x' ? 2 : 1), nullptr, e.size() > 1 && e[1] == 'x' ? 16 : 10));
            else { o.append(b + i, j - i + 1); }
            i = j;
        }
        return o;
    }
    std::unique_ptr<XmlElement> element(std::string& err) {
        p_++;   // '<'
        auto el = std::make_unique<XmlElement>();
        el->name = name();
        if (el->name.empty()) return fail(err, "empty element name");
        while (true) {                                   // attributes
            skip_ws();
            if (p_ >= n_) return fail(err, "unterminated start tag");
            if (starts("/>")) { p_ += 2; return el; }
            if (s_[p_] == '>') { p_++; break; }
            std::string k = name();
            if (k.empty()) return fail(err, "bad attribute");
            skip_ws();
            if (p_ >= n_ || s_[p_] != '=') return fail(err, "attribute without value");
            p_++;
            skip_ws();
            if (p_ >= n_ || (s_[p_] != '"' && s_[p_] != '\'')) return fail(err, "unquoted attribute");
            const char q = s_[p_++];
            size_t b = p_;
            while (p_ < n_ && s_[p_] != q) p_++;
            if (p_ >= n_) return fail(err, "unterminated attribute");
            el->attrs.emplace_back(k, unescape(s_ + b, p_ - b));
            p_++;
        }
        bool first_text = true;
        while (true) {                                   // content
            if (p_ >= n_) return fail(err, "unterminated element");
            if (starts("</")) {
                p_ += 2;
                std::string e = name();
                if (e != el->name) return fail(err, "mismatched end tag");
                skip_ws();
                if (p_ >= n_ || s_[p_] != '>') return fail(err, "bad end tag");
                p_++;
                return el;
            }
            if (starts("<!--")) { if (!skip_past("-->")) return fail(err, "unterminated comment"); continue; }
            if (starts("<![CDATA[")) {
                p_ += 9;
                size_t b = p_;
                if (!skip_past("]]>")) return fail(err, "unterminated CDATA");
                if (first_text && el->children.empty()) { el->text.append(s_ + b, p_ - 3 - b); el->has_text = true; }
                continue;
            }
            if (starts("<?")) { if (!skip_past("?>")) return fail(err, "unterminated PI"); continue; }
            if (s_[p_] == '<') {
                auto c = element(err);
                if (!c) return nullptr;
                el->children.push_back(std::move(c));
                first_text = false;
                continue;
            }
            size_t b = p_;
            while (p_ < n_ && s_[p_] != '<') p_++;
            if (first_text && el->children.empty()) { el->text += unescape(s_ + b, p_ - b); el->has_text = true; }
        }
    }
};

}  // namespace rtgh
