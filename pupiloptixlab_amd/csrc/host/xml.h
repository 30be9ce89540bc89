// xml.h — mitsuba-3 XML subset reader (replaces the reference's pugixml DFS,
// framework/resource/xml/parser.cpp:22-60, object.cpp:9-121, visitor.h:98-194).
//
// The reader produces the same Object tree the reference builds: one Object
// per bsdf/emitter/film/integrator/sensor/shape/texture/transform (+ lookat,
// rotate), properties for integer/string/float/rgb/point/matrix/scale/
// translate/boolean, `<default>` parameters substituted into `$name`
// attribute values, and `<ref id=...>` re-parenting an earlier object.
#pragma once

#include <map>
#include <memory>
#include <string>
#include <string_view>
#include <unordered_map>
#include <utility>
#include <vector>

namespace Pupil::resource::xml {

struct Property {
    std::string name;
    std::string value;
};

struct Object {
    std::string obj_name;  // element name (bsdf, shape, ...)
    std::string var_name;  // name="" attribute
    std::string id;
    std::string type;
    std::vector<Property> properties;
    std::vector<Object *> sub_object;

    std::string GetProperty(std::string_view name) const;
    Object *GetUniqueSubObject(std::string_view name) const;
    std::vector<Object *> GetSubObjects(std::string_view name) const;
    // sub-object whose name="" matches, else the property value (object.cpp:113-121)
    std::pair<Object *, std::string> GetParameter(std::string_view name) const;
};

class Parser {
public:
    // Returns the <scene> root or nullptr; error text in `error`.
    Object *LoadFromFile(const std::string &path, std::string *error = nullptr);
    Object *LoadFromString(const std::string &text, std::string *error = nullptr);

private:
    std::vector<std::unique_ptr<Object>> m_pool;
};

}  // namespace Pupil::resource::xml
