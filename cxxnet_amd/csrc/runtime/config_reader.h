// Config-language tokenizer for cxxnet .conf files.
//
// Grammar (behavioural parity with reference src/utils/config.h:20-141):
//   name = value          pairs separated by whitespace/newlines
//   # ...                 comment to end of line
//   "..."                 single-line string, backslash escapes the next char
//   '...'                 multi-line string, backslash escapes the next char
// A malformed pair (missing '=' or value) ends iteration, as in the reference.
#pragma once
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace cxxnet_rt {

using KVList = std::vector<std::pair<std::string, std::string>>;

class ConfigTokenizer {
 public:
  explicit ConfigTokenizer(std::string text) : text_(std::move(text)), pos_(0) {
    ch_ = get();
  }
  // Parse every pair in the text.
  KVList ParseAll() {
    KVList out;
    std::string name, eq, val;
    while (!end()) {
      bool nl = next_token(&name);
      (void)nl;
      if (name.empty() && end()) break;
      if (name == "=") break;
      if (next_token(&eq) || eq != "=") break;
      if (next_token(&val) || val == "=") break;
      out.emplace_back(name, val);
    }
    return out;
  }

 private:
  static constexpr int kEOF = -1;
  std::string text_;
  size_t pos_;
  int ch_;

  int get() { return pos_ < text_.size() ? static_cast<unsigned char>(text_[pos_++]) : kEOF; }
  bool end() const { return ch_ == kEOF; }

  void skip_line() {
    do { ch_ = get(); } while (ch_ != kEOF && ch_ != '\n' && ch_ != '\r');
  }
  void parse_str(std::string *tok, char quote, bool multiline) {
    while ((ch_ = get()) != kEOF) {
      if (ch_ == '\\') {
        int c = get();
        if (c != kEOF) *tok += static_cast<char>(c);
      } else if (ch_ == quote) {
        return;
      } else if (!multiline && (ch_ == '\r' || ch_ == '\n')) {
        throw std::runtime_error("ConfigReader: unterminated string");
      } else {
        *tok += static_cast<char>(ch_);
      }
    }
    throw std::runtime_error("ConfigReader: unterminated string");
  }
  // Returns true when a newline was crossed before any token character.
  bool next_token(std::string *tok) {
    tok->clear();
    bool new_line = false;
    while (ch_ != kEOF) {
      switch (ch_) {
        case '#':
          skip_line();
          new_line = true;
          break;
        case '"':
        case '\'':
          if (!tok->empty()) throw std::runtime_error("ConfigReader: token followed directly by string");
          parse_str(tok, static_cast<char>(ch_), ch_ == '\'');
          ch_ = get();
          return new_line;
        case '=':
          if (tok->empty()) {
            ch_ = get();
            *tok = "=";
          }
          return new_line;
        case '\r':
        case '\n':
          if (tok->empty()) new_line = true;
          [[fallthrough]];
        case '\t':
        case ' ':
          ch_ = get();
          if (!tok->empty()) return new_line;
          break;
        default:
          *tok += static_cast<char>(ch_);
          ch_ = get();
          break;
      }
    }
    return tok->empty();
  }
};

}  // namespace cxxnet_rt
