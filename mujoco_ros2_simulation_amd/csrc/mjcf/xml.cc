#include "xml.h"

#include <cctype>
#include <cstring>
#include <fstream>
#include <sstream>

namespace mrs {

namespace {

struct Cursor {
  const std::string& s;
  size_t i = 0;
  int line = 1;
  const std::string& origin;

  bool eof() const { return i >= s.size(); }
  char peek(size_t k = 0) const { return i + k < s.size() ? s[i + k] : '\0'; }
  char get() {
    char c = s[i++];
    if (c == '\n') ++line;
    return c;
  }
  bool starts(const char* p) const { return s.compare(i, std::strlen(p), p) == 0; }
  void skip(size_t n) { while (n-- && !eof()) get(); }
  void ws() { while (!eof() && std::isspace(static_cast<unsigned char>(peek()))) get(); }
  [[noreturn]] void fail(const std::string& msg) const {
    throw XmlError(origin + ":" + std::to_string(line) + ": XML error: " + msg);
  }
  void skip_until(const char* end) {
    while (!eof() && !starts(end)) get();
    if (eof()) fail(std::string("unterminated construct, expected '") + end + "'");
    skip(std::strlen(end));
  }
};

std::string decode_entities(const std::string& v) {
  if (v.find('&') == std::string::npos) return v;
  std::string out;
  for (size_t i = 0; i < v.size(); ++i) {
    if (v[i] != '&') { out += v[i]; continue; }
    size_t semi = v.find(';', i);
    if (semi == std::string::npos) { out += v[i]; continue; }
    std::string ent = v.substr(i + 1, semi - i - 1);
    if (ent == "lt") out += '<';
    else if (ent == "gt") out += '>';
    else if (ent == "amp") out += '&';
    else if (ent == "quot") out += '"';
    else if (ent == "apos") out += '\'';
    else { out += v.substr(i, semi - i + 1); }
    i = semi;
  }
  return out;
}

bool name_char(char c) {
  return std::isalnum(static_cast<unsigned char>(c)) || c == '_' || c == '-' || c == '.' || c == ':';
}

void skip_misc(Cursor& c) {
  for (;;) {
    c.ws();
    if (c.starts("<!--")) { c.skip_until("-->"); continue; }
    if (c.starts("<?")) { c.skip_until("?>"); continue; }
    if (c.starts("<!")) { c.skip_until(">"); continue; }
    break;
  }
}

std::unique_ptr<XmlElement> parse_element(Cursor& c) {
  if (c.peek() != '<') c.fail("expected '<'");
  c.get();
  auto e = std::make_unique<XmlElement>();
  e->line = c.line;
  while (!c.eof() && name_char(c.peek())) e->tag += c.get();
  if (e->tag.empty()) c.fail("empty tag name");
  for (;;) {
    c.ws();
    if (c.eof()) c.fail("unterminated tag <" + e->tag + ">");
    if (c.starts("/>")) { c.skip(2); return e; }
    if (c.peek() == '>') { c.get(); break; }
    std::string key;
    while (!c.eof() && name_char(c.peek())) key += c.get();
    if (key.empty()) c.fail("bad attribute in <" + e->tag + ">");
    c.ws();
    if (c.peek() != '=') c.fail("expected '=' after attribute " + key);
    c.get();
    c.ws();
    char q = c.peek();
    if (q != '"' && q != '\'') c.fail("attribute value must be quoted: " + key);
    c.get();
    std::string val;
    while (!c.eof() && c.peek() != q) val += c.get();
    if (c.eof()) c.fail("unterminated attribute value: " + key);
    c.get();
    for (auto& kv : e->attrs)
      if (kv.first == key) c.fail("duplicate attribute '" + key + "' in <" + e->tag + ">");
    e->attrs.emplace_back(key, decode_entities(val));
  }
  // content
  std::string text;
  for (;;) {
    while (!c.eof() && c.peek() != '<') text += c.get();
    if (c.eof()) c.fail("unterminated element <" + e->tag + ">");
    if (c.starts("<!--")) { c.skip_until("-->"); continue; }
    if (c.starts("<![CDATA[")) { c.skip_until("]]>"); continue; }
    if (c.starts("<?")) { c.skip_until("?>"); continue; }
    if (c.starts("</")) {
      c.skip(2);
      std::string tag;
      while (!c.eof() && name_char(c.peek())) tag += c.get();
      if (tag != e->tag) c.fail("mismatched closing tag </" + tag + "> for <" + e->tag + ">");
      c.ws();
      if (c.peek() != '>') c.fail("expected '>'");
      c.get();
      const auto b = text.find_first_not_of(" \t\r\n"), t = text.find_last_not_of(" \t\r\n");
      if (b != std::string::npos) e->text = decode_entities(text.substr(b, t - b + 1));
      return e;
    }
    e->children.push_back(parse_element(c));
  }
}

}  // namespace

std::unique_ptr<XmlElement> xml_parse(const std::string& text, const std::string& origin) {
  Cursor c{text, 0, 1, origin};
  skip_misc(c);
  if (c.eof()) c.fail("empty document");
  auto root = parse_element(c);
  skip_misc(c);
  if (!c.eof()) c.fail("trailing content after root element");
  return root;
}

std::string read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw XmlError("could not open file '" + path + "'");
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

}  // namespace mrs
