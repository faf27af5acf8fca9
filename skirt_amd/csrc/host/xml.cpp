#include "xml.hpp"

#include <fstream>
#include <sstream>
#include <stdexcept>

namespace skirt {

bool XmlElement::has(const std::string& key) const {
    for (auto& kv : attributes)
        if (kv.first == key) return true;
    return false;
}

std::string XmlElement::get(const std::string& key, const std::string& def) const {
    for (auto& kv : attributes)
        if (kv.first == key) return kv.second;
    return def;
}

const XmlElement* XmlElement::child(const std::string& n) const {
    for (auto& c : children)
        if (c->name == n) return c.get();
    return nullptr;
}

const XmlElement* XmlElement::item(const std::string& prop) const {
    const XmlElement* p = child(prop);
    if (!p || p->children.empty()) return nullptr;
    return p->children.front().get();
}

std::vector<const XmlElement*> XmlElement::items(const std::string& prop) const {
    std::vector<const XmlElement*> out;
    const XmlElement* p = child(prop);
    if (p)
        for (auto& c : p->children) out.push_back(c.get());
    return out;
}

namespace {

class Parser {
public:
    explicit Parser(const std::string& s) : s_(s) {}

    std::unique_ptr<XmlElement> document() {
        skipMisc();
        if (pos_ >= s_.size() || s_[pos_] != '<') fail("expected root element");
        auto root = element();
        skipMisc();
        if (pos_ != s_.size()) fail("trailing content after root element");
        return root;
    }

private:
    const std::string& s_;
    size_t pos_ = 0;

    [[noreturn]] void fail(const std::string& msg) const {
        size_t line = 1;
        for (size_t i = 0; i < pos_ && i < s_.size(); ++i)
            if (s_[i] == '\n') ++line;
        throw std::runtime_error("XML parse error at line " + std::to_string(line) + ": " + msg);
    }

    bool starts(const char* lit) const { return s_.compare(pos_, std::char_traits<char>::length(lit), lit) == 0; }

    void skipWs() {
        while (pos_ < s_.size() && (s_[pos_] == ' ' || s_[pos_] == '\t' || s_[pos_] == '\n' || s_[pos_] == '\r'))
            ++pos_;
    }

    // skips whitespace, text, comments, processing instructions and DOCTYPE
    void skipMisc() {
        while (true) {
            while (pos_ < s_.size() && s_[pos_] != '<') ++pos_;
            if (pos_ >= s_.size()) return;
            if (starts("<!--")) {
                size_t e = s_.find("-->", pos_ + 4);
                if (e == std::string::npos) fail("unterminated comment");
                pos_ = e + 3;
            } else if (starts("<?")) {
                size_t e = s_.find("?>", pos_ + 2);
                if (e == std::string::npos) fail("unterminated processing instruction");
                pos_ = e + 2;
            } else if (starts("<!")) {
                size_t e = s_.find('>', pos_ + 2);
                if (e == std::string::npos) fail("unterminated declaration");
                pos_ = e + 1;
            } else {
                return;
            }
        }
    }

    std::string name() {
        size_t b = pos_;
        while (pos_ < s_.size()) {
            char c = s_[pos_];
            if (c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '/' || c == '>' || c == '=') break;
            ++pos_;
        }
        if (pos_ == b) fail("expected a name");
        return s_.substr(b, pos_ - b);
    }

    static std::string unescape(const std::string& v) {
        std::string out;
        out.reserve(v.size());
        for (size_t i = 0; i < v.size(); ++i) {
            if (v[i] != '&') { out += v[i]; continue; }
            size_t e = v.find(';', i);
            std::string ent = (e == std::string::npos) ? "" : v.substr(i + 1, e - i - 1);
            if (ent == "amp") out += '&';
            else if (ent == "lt") out += '<';
            else if (ent == "gt") out += '>';
            else if (ent == "quot") out += '"';
            else if (ent == "apos") out += '\'';
            else { out += '&'; continue; }
            i = e;
        }
        return out;
    }

    std::unique_ptr<XmlElement> element() {
        ++pos_;  // '<'
        auto el = std::make_unique<XmlElement>();
        el->name = name();
        while (true) {
            skipWs();
            if (pos_ >= s_.size()) fail("unterminated start tag");
            if (starts("/>")) { pos_ += 2; return el; }
            if (s_[pos_] == '>') { ++pos_; break; }
            std::string key = name();
            skipWs();
            if (pos_ >= s_.size() || s_[pos_] != '=') fail("expected '=' after attribute " + key);
            ++pos_;
            skipWs();
            if (pos_ >= s_.size() || (s_[pos_] != '"' && s_[pos_] != '\'')) fail("expected quoted attribute value");
            char q = s_[pos_++];
            size_t e = s_.find(q, pos_);
            if (e == std::string::npos) fail("unterminated attribute value");
            el->attributes.emplace_back(key, unescape(s_.substr(pos_, e - pos_)));
            pos_ = e + 1;
        }
        // content
        while (true) {
            skipMisc();
            if (pos_ >= s_.size()) fail("unterminated element " + el->name);
            if (starts("</")) {
                pos_ += 2;
                std::string n = name();
                if (n != el->name) fail("mismatched end tag " + n + " for " + el->name);
                skipWs();
                if (pos_ >= s_.size() || s_[pos_] != '>') fail("malformed end tag");
                ++pos_;
                return el;
            }
            el->children.push_back(element());
        }
    }
};

}  // namespace

std::unique_ptr<XmlElement> parseXmlString(const std::string& text) {
    Parser p(text);
    return p.document();
}

std::unique_ptr<XmlElement> parseXmlFile(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open ski file " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    return parseXmlString(ss.str());
}

}  // namespace skirt
