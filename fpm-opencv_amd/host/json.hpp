// json.hpp -- small JSON DOM for the dataset-config contract.
//
// The reference parses its dataset JSON with jsoncpp 1.6.5
// (include/jsoncpp.cpp, Json::Reader::parse at fpmMain.cpp:512-515) and
// IGNORES the parse result.  Two shipped configs (dataset_dogStomach.json,
// dataset_cellScope.json) end their holeCoordinates array with a trailing
// comma; jsoncpp then appends one null element, abandons the rest of the
// document and keeps the partial tree, which the reference goes on to use
// (SURVEY.md 8(c)).  This reader reproduces that recovery: on the first
// syntax error the values built so far are kept, a null is left in the slot
// being parsed, and parsing stops.  Accessors follow jsoncpp's conversion
// rules (asInt truncates reals, asBool of a number is != 0, ...).
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace fpmhost {

class Json {
   public:
    enum Type { Null, Bool, Int, Real, String, Array, Object };

    Json() = default;
    static Json make_bool(bool b);
    static Json make_int(int64_t v);
    static Json make_real(double v);
    static Json make_string(std::string s);
    static Json make_array();
    static Json make_object();

    Type type() const { return type_; }
    bool is_null() const { return type_ == Null; }
    bool is_array() const { return type_ == Array; }
    bool is_object() const { return type_ == Object; }
    size_t size() const;

    // jsoncpp-style accessors (Json::Value::asInt/asDouble/...)
    int as_int() const;      // throws std::runtime_error where jsoncpp throws
    double as_double() const;
    float as_float() const { return (float)as_double(); }
    bool as_bool() const;
    std::string as_string() const;

    // get(key, default): member if present (object only), else default
    const Json &get(const std::string &key, const Json &dflt) const;
    bool has(const std::string &key) const;
    // array element; out of range or non-array -> a shared null (like a const
    // jsoncpp access would; the reference's non-const access on a null value
    // throws, which callers check via is_array()).
    const Json &at(size_t i) const;

    // set (or add) an object member; converts null to an object
    void set(const std::string &key, Json v);

    std::vector<Json> &items() { return arr_; }
    const std::vector<Json> &items() const { return arr_; }
    std::vector<std::pair<std::string, Json>> &members() { return obj_; }
    const std::vector<std::pair<std::string, Json>> &members() const { return obj_; }

   private:
    Type type_ = Null;
    bool b_ = false;
    int64_t i_ = 0;
    double d_ = 0.0;
    std::string s_;
    std::vector<Json> arr_;
    std::vector<std::pair<std::string, Json>> obj_;
};

struct JsonParseResult {
    Json root;
    bool ok = true;          // false when a syntax error stopped the parse
    std::string error;       // description of that error
    size_t error_offset = 0;
};

JsonParseResult parse_json(const std::string &text);
bool read_file(const std::string &path, std::string *out);

}  // namespace fpmhost
