#include "xml.h"

#include <algorithm>
#include <cstdlib>
#include <string_view>

namespace ksa {

namespace {

void put_utf8(std::string* s, unsigned long cp) {
  if (cp < 0x80) {
    s->push_back(static_cast<char>(cp));
  } else if (cp < 0x800) {
    s->push_back(static_cast<char>(0xC0 | (cp >> 6)));
    s->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  } else if (cp < 0x10000) {
    s->push_back(static_cast<char>(0xE0 | (cp >> 12)));
    s->push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
    s->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  } else {
    s->push_back(static_cast<char>(0xF0 | (cp >> 18)));
    s->push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
    s->push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
    s->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  }
}

// Does doc[b, e) -- an element name, possibly namespace-prefixed -- have the local name `tag`?
// Compared in place: no substring per tag scanned.
bool local_name_is(const std::string& doc, size_t b, size_t e, std::string_view tag) {
  for (size_t k = b; k < e; ++k)
    if (doc[k] == ':') b = k + 1;  // the prefix ends at the (last) colon
  return e - b == tag.size() && doc.compare(b, e - b, tag) == 0;
}

// Walks the start tags at or after `pos` (their '<' before `to`) and records, for each of the
// `n` tags, the first start tag with that local name: starts[i] = the offset just past its '>'
// (npos if none), self_closing[i] for <x/>. Stops once all are found. The walk visits the same
// positions whatever the tags are, so looking for several tags in one walk finds exactly what
// one walk per tag would.
void find_starts(const std::string& doc, const std::string_view* tags, size_t n, size_t pos,
                 size_t to, size_t* starts, bool* self_closing) {
  size_t left = n;
  for (size_t i = 0; i < n; ++i) starts[i] = std::string::npos;
  while (left > 0) {
    size_t lt = doc.find('<', pos);
    if (lt == std::string::npos || lt >= to) return;
    size_t p = lt + 1;
    if (p < doc.size() && (doc[p] == '/' || doc[p] == '?' || doc[p] == '!')) {
      pos = p;
      continue;
    }
    size_t name_end = p;
    while (name_end < doc.size() && doc[name_end] != '>' && doc[name_end] != ' ' &&
           doc[name_end] != '/' && doc[name_end] != '\t' && doc[name_end] != '\n' &&
           doc[name_end] != '\r')
      ++name_end;
    size_t gt = doc.find('>', name_end);
    if (gt == std::string::npos) return;
    for (size_t i = 0; i < n; ++i) {
      if (starts[i] == std::string::npos && local_name_is(doc, p, name_end, tags[i])) {
        starts[i] = gt + 1;
        self_closing[i] = gt > 0 && doc[gt - 1] == '/';
        --left;
      }
    }
    pos = gt + 1;
  }
}

// The next start tag whose local name equals `tag` at or after `pos` (before `to`): the offset
// just past its '>', or npos. *self_closing set for <x/>.
size_t find_start(const std::string& doc, std::string_view tag, size_t pos, size_t to,
                  bool* self_closing) {
  size_t start;
  find_starts(doc, &tag, 1, pos, to, &start, self_closing);
  return start;
}

size_t find_end(const std::string& doc, std::string_view tag, size_t pos, size_t to) {
  while (true) {
    size_t lt = doc.find("</", pos);
    if (lt == std::string::npos || lt >= to) return std::string::npos;
    size_t p = lt + 2;
    size_t gt = doc.find('>', p);
    if (gt == std::string::npos) return std::string::npos;
    size_t e = gt;
    while (e > p && (doc[e - 1] == ' ' || doc[e - 1] == '\t')) --e;
    if (local_name_is(doc, p, e, tag)) return lt;
    pos = gt + 1;
  }
}

}  // namespace

std::string xml_unescape(const std::string& s) {
  if (s.find('&') == std::string::npos) return s;
  std::string out;
  out.reserve(s.size());
  size_t i = 0;
  while (i < s.size()) {
    if (s[i] != '&') {
      out.push_back(s[i++]);
      continue;
    }
    size_t semi = s.find(';', i);
    if (semi == std::string::npos || semi - i > 12) {
      out.push_back(s[i++]);
      continue;
    }
    std::string ent = s.substr(i + 1, semi - i - 1);
    if (ent == "amp") out.push_back('&');
    else if (ent == "lt") out.push_back('<');
    else if (ent == "gt") out.push_back('>');
    else if (ent == "quot") out.push_back('"');
    else if (ent == "apos") out.push_back('\'');
    else if (!ent.empty() && ent[0] == '#') {
      unsigned long cp = (ent.size() > 1 && (ent[1] == 'x' || ent[1] == 'X'))
                             ? std::strtoul(ent.c_str() + 2, nullptr, 16)
                             : std::strtoul(ent.c_str() + 1, nullptr, 10);
      put_utf8(&out, cp);
    } else {
      out.append(s, i, semi - i + 1);
    }
    i = semi + 1;
  }
  return out;
}

std::string xml_escape(const std::string& s) {
  std::string out;
  out.reserve(s.size());
  for (char c : s) {
    switch (c) {
      case '&': out += "&amp;"; break;
      case '<': out += "&lt;"; break;
      case '>': out += "&gt;"; break;
      case '"': out += "&quot;"; break;
      case '\'': out += "&apos;"; break;
      default: out.push_back(c);
    }
  }
  return out;
}

namespace {

// The text of the element whose start tag ends at `start` (xml_first_text after the start tag).
std::string text_from(const std::string& doc, std::string_view tag, size_t start, bool self_closing,
                      size_t to) {
  if (self_closing) return "";
  size_t end = find_end(doc, tag, start, to);
  if (end == std::string::npos) end = to;
  // [start, start + n): what doc.substr(start, end - start) keeps (the start tag can end past
  // `to`, then end < start and the text runs to the end of doc).
  const size_t n = std::min(end - start, doc.size() - start);
  // CDATA sections are passed through verbatim.
  if (n >= 12 && doc.compare(start, 9, "<![CDATA[") == 0 && doc.compare(start + n - 3, 3, "]]>") == 0)
    return doc.substr(start + 9, n - 12);
  if (std::char_traits<char>::find(doc.data() + start, n, '&') == nullptr) return doc.substr(start, n);
  return xml_unescape(doc.substr(start, n));
}

}  // namespace

std::string xml_first_text(const std::string& doc, const std::string& tag, bool* found,
                           size_t from, size_t to) {
  if (to > doc.size()) to = doc.size();
  bool self_closing = false;
  size_t start = find_start(doc, tag, from, to, &self_closing);
  if (found) *found = start != std::string::npos;
  if (start == std::string::npos) return "";
  return text_from(doc, tag, start, self_closing, to);
}

std::vector<std::pair<std::string, std::string>> xml_sqs_attributes(const std::string& doc) {
  std::vector<std::pair<std::string, std::string>> out;
  out.reserve(4);
  size_t pos = 0;
  while (true) {
    bool sc = false;
    size_t start = find_start(doc, "Attribute", pos, doc.size(), &sc);
    if (start == std::string::npos) break;
    if (sc) {
      pos = start;
      continue;
    }
    size_t end = find_end(doc, "Attribute", start, doc.size());
    if (end == std::string::npos) break;
    // xml_first_text(Name) and xml_first_text(Value) over [start, end), in one walk.
    static constexpr std::string_view kTags[2] = {"Name", "Value"};
    size_t at[2];
    bool sc2[2] = {false, false};
    find_starts(doc, kTags, 2, start, end, at, sc2);
    if (at[0] != std::string::npos)
      out.emplace_back(text_from(doc, kTags[0], at[0], sc2[0], end),
                       at[1] == std::string::npos ? std::string() : text_from(doc, kTags[1], at[1], sc2[1], end));
    pos = end + 1;
  }
  return out;
}

}  // namespace ksa
