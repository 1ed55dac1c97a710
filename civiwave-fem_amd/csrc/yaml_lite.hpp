// yaml_lite.hpp -- the YAML subset CiviWave scenarios use (yaml-cpp is not available offline).
//
// Supported: block mappings and block sequences by indentation (sequences may sit at their parent
// key's indent), "- key: value" sequence items that open a mapping, flow sequences / mappings
// ([a, [b, c]], {k: v}) anywhere a value goes, plain / single- / double-quoted scalars, '#'
// comments, null (~, null, empty). Scalar conversions follow yaml-cpp's convert<> rules for the
// types the config reads (double incl. .inf/.nan, bool y/yes/true/on..., unsigned rejects '-').
// Errors are thrown as yl::Error with yaml-cpp-like texts ("bad conversion", "invalid node; first
// invalid key: \"E\"") and 1-based line / column.
#pragma once

#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace yl
{

struct Error : std::runtime_error
{
    using std::runtime_error::runtime_error;
};

struct Node
{
    enum Kind
    {
        Undefined,  // a missing key / out-of-range index (yaml-cpp's zombie node)
        Null,
        Scalar,
        Seq,
        Map
    };
    Kind kind = Undefined;
    std::string text;  // scalar text
    bool quoted = false;
    std::vector<Node> items;                         // Seq
    std::vector<std::pair<std::string, Node>> map;  // Map, file order
    int line = 0, col = 0;
    std::string missing_key;  // Undefined: the key that was looked up

    bool defined() const { return kind != Undefined; }
    bool is_null() const { return kind == Null; }
    bool is_scalar() const { return kind == Scalar; }
    bool is_seq() const { return kind == Seq; }
    bool is_map() const { return kind == Map; }
    size_t size() const { return kind == Seq ? items.size() : kind == Map ? map.size() : 0; }

    const Node &operator[](const std::string &key) const
    {
        if (kind == Map)
            for (const auto &kv : map)
                if (kv.first == key)
                    return kv.second;
        static thread_local Node zombie;
        zombie = Node{};
        zombie.missing_key = key;
        zombie.line = line;
        zombie.col = col;
        return zombie;
    }
    const Node &operator[](size_t i) const
    {
        if (kind == Seq && i < items.size())
            return items[i];
        static thread_local Node zombie;
        zombie = Node{};
        zombie.missing_key = std::to_string(i);
        return zombie;
    }

    [[noreturn]] void bad() const
    {
        if (kind == Undefined)
            throw Error("invalid node; first invalid key: \"" + missing_key + "\"");
        throw Error("yaml-cpp: error at line " + std::to_string(line) + ", column " + std::to_string(col) +
                    ": bad conversion");
    }
    std::string as_string() const
    {
        if (kind != Scalar)
            bad();
        return text;
    }
    double as_double() const
    {
        if (kind != Scalar || text.empty())
            bad();
        const std::string &t = text;
        if (t == ".inf" || t == ".Inf" || t == ".INF" || t == "+.inf" || t == "+.Inf" || t == "+.INF")
            return INFINITY;
        if (t == "-.inf" || t == "-.Inf" || t == "-.INF")
            return -INFINITY;
        if (t == ".nan" || t == ".NaN" || t == ".NAN")
            return NAN;
        char *end = nullptr;
        errno = 0;
        const double v = std::strtod(t.c_str(), &end);
        if (end == t.c_str() || *end != '\0' || t[0] == ' ' || std::isinf(v) || std::isnan(v))
            bad();
        return v;
    }
    bool as_bool() const
    {
        if (kind != Scalar)
            bad();
        static const char *yes[] = {"y", "Y", "yes", "Yes", "YES", "true", "True", "TRUE", "on", "On", "ON"};
        static const char *no[] = {"n", "N", "no", "No", "NO", "false", "False", "FALSE", "off", "Off", "OFF"};
        for (const char *s : yes)
            if (text == s)
                return true;
        for (const char *s : no)
            if (text == s)
                return false;
        bad();
    }
    uint32_t as_u32() const
    {
        if (kind != Scalar || text.empty() || text[0] == '-')
            bad();
        char *end = nullptr;
        errno = 0;
        const unsigned long long v = std::strtoull(text.c_str(), &end, 0);
        if (end == text.c_str() || *end != '\0' || errno == ERANGE || v > 0xFFFFFFFFull)
            bad();
        return (uint32_t)v;
    }
};

namespace detail
{

struct Line
{
    int number;  // 1-based
    int indent;
    std::string text;  // content after indentation, comment stripped, right-trimmed
};

inline std::string rtrim(std::string s)
{
    while (!s.empty() && (s.back() == ' ' || s.back() == '\t' || s.back() == '\r'))
        s.pop_back();
    return s;
}

// drop a '#' comment that starts the line or follows whitespace, outside quotes
inline std::string strip_comment(const std::string &s)
{
    char q = 0;
    for (size_t i = 0; i < s.size(); ++i)
    {
        const char c = s[i];
        if (q)
        {
            if (c == q)
                q = 0;
            continue;
        }
        if (c == '"' || c == '\'')
            q = c;
        else if (c == '#' && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '\t'))
            return s.substr(0, i);
    }
    return s;
}

class Parser
{
public:
    explicit Parser(const std::string &src)
    {
        size_t pos = 0;
        int number = 0;
        while (pos <= src.size())
        {
            size_t nl = src.find('\n', pos);
            if (nl == std::string::npos)
                nl = src.size();
            std::string raw = src.substr(pos, nl - pos);
            ++number;
            pos = nl + 1;
            if (raw.rfind("---", 0) == 0 || raw.rfind("...", 0) == 0)
                continue;
            std::string t = rtrim(strip_comment(raw));
            size_t ind = 0;
            while (ind < t.size() && t[ind] == ' ')
                ++ind;
            if (ind == t.size())
                continue;
            if (t[ind] == '\t')
                throw Error("yaml-cpp: error at line " + std::to_string(number) + ", column " +
                            std::to_string(ind + 1) + ": illegal tab when looking for indentation");
            lines_.push_back(Line{number, (int)ind, t.substr(ind)});
            if (nl == src.size())
                break;
        }
    }

    Node document()
    {
        if (lines_.empty())
        {
            Node n;
            n.kind = Node::Null;
            return n;
        }
        Node n = block(lines_[0].indent);
        if (i_ < lines_.size())
            fail(lines_[i_], 1, "end of map not found");
        return n;
    }

private:
    std::vector<Line> lines_;
    size_t i_ = 0;

    [[noreturn]] static void fail(const Line &l, int col, const std::string &what)
    {
        throw Error("yaml-cpp: error at line " + std::to_string(l.number) + ", column " + std::to_string(col) +
                    ": " + what);
    }

    static bool is_seq_item(const std::string &t) { return t == "-" || t.rfind("- ", 0) == 0; }

    // position of the ':' that ends a plain / quoted mapping key on this line, or npos
    static size_t key_colon(const std::string &t)
    {
        if (t.empty() || t[0] == '[' || t[0] == '{')
            return std::string::npos;
        size_t i = 0;
        if (t[0] == '"' || t[0] == '\'')
        {
            const char q = t[0];
            i = t.find(q, 1);
            if (i == std::string::npos)
                return std::string::npos;
            ++i;
            return (i < t.size() && t[i] == ':' && (i + 1 == t.size() || t[i + 1] == ' ')) ? i : std::string::npos;
        }
        for (; i < t.size(); ++i)
            if (t[i] == ':' && (i + 1 == t.size() || t[i + 1] == ' '))
                return i;
        return std::string::npos;
    }

    static std::string unquote_key(const std::string &k)
    {
        if (k.size() >= 2 && (k[0] == '"' || k[0] == '\'') && k.back() == k[0])
            return k.substr(1, k.size() - 2);
        return k;
    }

    // a block node whose first line is lines_[i_] at indentation `ind`
    Node block(int ind)
    {
        const Line &first = lines_[i_];
        if (is_seq_item(first.text))
            return sequence(ind);
        if (key_colon(first.text) != std::string::npos)
            return mapping(ind);
        ++i_;
        return inline_value(first, first.text, first.indent + 1);
    }

    Node sequence(int ind)
    {
        Node n;
        n.kind = Node::Seq;
        n.line = lines_[i_].number;
        n.col = ind + 1;
        while (i_ < lines_.size() && lines_[i_].indent == ind && is_seq_item(lines_[i_].text))
        {
            Line &l = lines_[i_];
            std::string rest = l.text.size() > 1 ? l.text.substr(2) : std::string();
            size_t lead = 0;
            while (lead < rest.size() && rest[lead] == ' ')
                ++lead;
            rest = rest.substr(lead);
            if (rest.empty())
            {
                ++i_;
                if (i_ < lines_.size() && lines_[i_].indent > ind)
                    n.items.push_back(block(lines_[i_].indent));
                else
                {
                    Node z;
                    z.kind = Node::Null;
                    n.items.push_back(z);
                }
                continue;
            }
            const int col = ind + 2 + (int)lead;
            if (is_seq_item(rest) || key_colon(rest) != std::string::npos)
            {
                // "- key: v" / "- - x": the item is a block node starting at this column
                l.indent = col;
                l.text = rest;
                n.items.push_back(block(col));
                continue;
            }
            ++i_;
            n.items.push_back(inline_value(l, rest, col + 1));
        }
        return n;
    }

    Node mapping(int ind)
    {
        Node n;
        n.kind = Node::Map;
        n.line = lines_[i_].number;
        n.col = ind + 1;
        while (i_ < lines_.size() && lines_[i_].indent == ind)
        {
            const Line &l = lines_[i_];
            const size_t c = key_colon(l.text);
            if (c == std::string::npos)
                fail(l, ind + 1, is_seq_item(l.text) ? "end of map not found" : "illegal map value");
            std::string key = unquote_key(rtrim(l.text.substr(0, c)));
            for (const auto &kv : n.map)
                if (kv.first == key)
                    fail(l, ind + 1, "duplicate key \"" + key + "\"");
            std::string rest = c + 1 < l.text.size() ? l.text.substr(c + 1) : std::string();
            size_t lead = 0;
            while (lead < rest.size() && rest[lead] == ' ')
                ++lead;
            rest = rest.substr(lead);
            ++i_;
            Node v;
            if (rest.empty())
            {
                if (i_ < lines_.size() && lines_[i_].indent > ind)
                    v = block(lines_[i_].indent);
                else if (i_ < lines_.size() && lines_[i_].indent == ind && is_seq_item(lines_[i_].text))
                    v = sequence(ind);  // "key:\n- a" (sequence at the key's indentation)
                else
                {
                    v.kind = Node::Null;
                    v.line = l.number;
                    v.col = (int)(ind + c + 2);
                }
            }
            else
                v = inline_value(l, rest, (int)(ind + c + 2 + lead));
            n.map.emplace_back(std::move(key), std::move(v));
        }
        return n;
    }

    Node inline_value(const Line &l, const std::string &s, int col)
    {
        size_t p = 0;
        Node v = flow(l, s, p, col, false);
        while (p < s.size() && s[p] == ' ')
            ++p;
        if (p != s.size())
            fail(l, col + (int)p, "unexpected characters after value");
        return v;
    }

    // flow value starting at s[p]; in_flow: ',' ']' '}' end plain scalars
    Node flow(const Line &l, const std::string &s, size_t &p, int col, bool in_flow)
    {
        while (p < s.size() && s[p] == ' ')
            ++p;
        Node n;
        n.line = l.number;
        n.col = col + (int)p;
        if (p < s.size() && s[p] == '[')
        {
            n.kind = Node::Seq;
            ++p;
            for (;;)
            {
                while (p < s.size() && s[p] == ' ')
                    ++p;
                if (p >= s.size())
                    fail(l, col + (int)p, "end of sequence flow not found");
                if (s[p] == ']')
                {
                    ++p;
                    break;
                }
                n.items.push_back(flow(l, s, p, col, true));
                while (p < s.size() && s[p] == ' ')
                    ++p;
                if (p < s.size() && s[p] == ',')
                    ++p;
                else if (p < s.size() && s[p] == ']')
                {
                    ++p;
                    break;
                }
                else
                    fail(l, col + (int)p, "end of sequence flow not found");
            }
            return n;
        }
        if (p < s.size() && s[p] == '{')
        {
            n.kind = Node::Map;
            ++p;
            for (;;)
            {
                while (p < s.size() && s[p] == ' ')
                    ++p;
                if (p >= s.size())
                    fail(l, col + (int)p, "end of map flow not found");
                if (s[p] == '}')
                {
                    ++p;
                    break;
                }
                Node k = scalar(l, s, p, col, true, true);
                while (p < s.size() && s[p] == ' ')
                    ++p;
                if (p >= s.size() || s[p] != ':')
                    fail(l, col + (int)p, "end of map flow not found");
                ++p;
                Node v = flow(l, s, p, col, true);
                n.map.emplace_back(k.text, std::move(v));
                while (p < s.size() && s[p] == ' ')
                    ++p;
                if (p < s.size() && s[p] == ',')
                    ++p;
                else if (p < s.size() && s[p] == '}')
                {
                    ++p;
                    break;
                }
                else
                    fail(l, col + (int)p, "end of map flow not found");
            }
            return n;
        }
        return scalar(l, s, p, col, in_flow, false);
    }

    Node scalar(const Line &l, const std::string &s, size_t &p, int col, bool in_flow, bool as_key)
    {
        Node n;
        n.line = l.number;
        n.col = col + (int)p;
        n.kind = Node::Scalar;
        if (p < s.size() && (s[p] == '"' || s[p] == '\''))
        {
            const char q = s[p++];
            std::string out;
            for (;;)
            {
                if (p >= s.size())
                    fail(l, n.col, "end of quoted scalar not found");
                const char c = s[p++];
                if (q == '\'' && c == '\'' && p < s.size() && s[p] == '\'')
                {
                    out.push_back('\'');
                    ++p;
                    continue;
                }
                if (c == q)
                    break;
                if (q == '"' && c == '\\' && p < s.size())
                {
                    const char e = s[p++];
                    out.push_back(e == 'n' ? '\n' : e == 't' ? '\t' : e);
                    continue;
                }
                out.push_back(c);
            }
            n.text = out;
            n.quoted = true;
            return n;
        }
        const size_t b = p;
        while (p < s.size())
        {
            const char c = s[p];
            if (in_flow && (c == ',' || c == ']' || c == '}'))
                break;
            if (as_key && c == ':' && (p + 1 == s.size() || s[p + 1] == ' '))
                break;
            ++p;
        }
        n.text = rtrim(s.substr(b, p - b));
        if (!as_key && (n.text.empty() || n.text == "~" || n.text == "null" || n.text == "Null" || n.text == "NULL"))
        {
            n.kind = Node::Null;
            n.text.clear();
        }
        return n;
    }
};

}  // namespace detail

inline Node parse(const std::string &text)
{
    detail::Parser p(text);
    return p.document();
}

}  // namespace yl
