// Minimal XML DOM for MJCF files (no tinyxml2 in this image; the reference links tinyxml2 for the
// keyframe override file, src/mujoco_system_interface.cpp:1552-1575, and MuJoCo's own parser reads
// the MJCF).  Supports elements, attributes, comments, declarations, CDATA-free text and the five
// predefined entities.  Element text is kept (URDF <param> values).  Errors carry a line number.
#pragma once

#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace mrs {

struct XmlElement {
  std::string tag;
  std::vector<std::pair<std::string, std::string>> attrs;
  std::vector<std::unique_ptr<XmlElement>> children;
  std::string text;  // concatenated character data, whitespace-trimmed, entities decoded
  int line = 0;

  const std::string* attr(const std::string& key) const {
    for (auto& kv : attrs)
      if (kv.first == key) return &kv.second;
    return nullptr;
  }
  void set_attr(const std::string& key, const std::string& val) {
    for (auto& kv : attrs)
      if (kv.first == key) { kv.second = val; return; }
    attrs.emplace_back(key, val);
  }
  std::unique_ptr<XmlElement> clone() const {
    auto e = std::make_unique<XmlElement>();
    e->tag = tag; e->attrs = attrs; e->text = text; e->line = line;
    for (auto& c : children) e->children.push_back(c->clone());
    return e;
  }
};

struct XmlError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// Parse a whole document; returns the root element.  `origin` is used in error messages.
std::unique_ptr<XmlElement> xml_parse(const std::string& text, const std::string& origin);

// Read a file into a string (throws XmlError if it cannot be read).
std::string read_file(const std::string& path);

}  // namespace mrs
