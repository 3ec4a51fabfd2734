// Tiny XML scanner for AWS Query-protocol responses.
//
// aws-sdk-go v1.35.35 (/root/reference/go.mod:6) speaks the SQS Query protocol: the
// GetQueueAttributes result is a list of <Attribute><Name/><Value/></Attribute> elements and
// failures are <ErrorResponse><Error><Code/><Message/></Error><RequestId/></ErrorResponse>.
// Those are the only shapes this project reads, so a streaming element scanner (no DTDs,
// no namespaces beyond ignoring prefixes) is all that is needed.
#pragma once

#include <string>
#include <utility>
#include <vector>

namespace ksa {

// Decodes the five predefined entities plus &#N; / &#xN; references.
std::string xml_unescape(const std::string& s);
std::string xml_escape(const std::string& s);

// Text content of the first <tag>...</tag> (namespace prefix ignored) inside [from, to)
// of `doc`; `found` reports presence. Nested markup inside the element is not expected.
std::string xml_first_text(const std::string& doc, const std::string& tag, bool* found,
                           size_t from = 0, size_t to = std::string::npos);

// All (Name, Value) pairs of <Attribute> elements, in document order.
std::vector<std::pair<std::string, std::string>> xml_sqs_attributes(const std::string& doc);

}  // namespace ksa
