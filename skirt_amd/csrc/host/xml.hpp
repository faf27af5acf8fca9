// Minimal XML DOM for SKIRT .ski parameter files.
//
// A .ski file is an XML tree in which an element names a SimulationItem class, an attribute holds a
// scalar property (optionally with a unit string) and a lowercase child element holds a compound
// property whose own children are the item(s) assigned to it
// (reference: doc/Part 1 - User Guide/SKIRT/ski files.txt:1-75, Discover/XmlHierarchyCreator.cpp:70-163).
// Only what that format uses is supported: elements, attributes, comments, the XML declaration and the
// five predefined entities. Text content is ignored.
#pragma once

#include <map>
#include <memory>
#include <string>
#include <vector>

namespace skirt {

struct XmlElement {
    std::string name;
    std::vector<std::pair<std::string, std::string>> attributes;
    std::vector<std::unique_ptr<XmlElement>> children;

    bool has(const std::string& key) const;
    // returns the attribute value, or `def` when absent
    std::string get(const std::string& key, const std::string& def = "") const;
    // first child element with the given name, or nullptr
    const XmlElement* child(const std::string& name) const;
    // the single item element held by compound property `prop` (e.g. <dustGrid type="..."><OctTreeDustGrid/></dustGrid>)
    const XmlElement* item(const std::string& prop) const;
    // all item elements held by a list property (e.g. <components type="StellarComp"> ... </components>)
    std::vector<const XmlElement*> items(const std::string& prop) const;
};

// Parses the file; throws std::runtime_error with a line number on malformed input.
std::unique_ptr<XmlElement> parseXmlFile(const std::string& path);
std::unique_ptr<XmlElement> parseXmlString(const std::string& text);

}  // namespace skirt
