// Minimal flag parser shared by the command-line apps.  Positional `M N`
// stays compatible with the reference (`prog [M N]`, atoi, default 40 40:
// stage2-mpi/poisson_mpi_decomp.cpp:470-474); everything else is a flag with
// a PE_* environment mirror (e.g. --tol ↔ PE_TOL).
#pragma once

#include <cstdlib>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

namespace pe {

class Args {
 public:
  Args(int argc, char** argv) {
    for (int i = 1; i < argc; ++i) {
      std::string a = argv[i];
      if (a.rfind("--", 0) == 0) {
        std::string key = a.substr(2), val = "1";
        const auto eq = key.find('=');
        if (eq != std::string::npos) {
          val = key.substr(eq + 1);
          key = key.substr(0, eq);
        } else if (i + 1 < argc && std::string(argv[i + 1]).rfind("--", 0) != 0 &&
                   !is_bool_flag(key)) {
          val = argv[++i];
        }
        kv_[key] = val;
      } else {
        pos_.push_back(a);
      }
    }
  }
  std::string get(const std::string& k, const std::string& def) const {
    auto it = kv_.find(k);
    if (it != kv_.end()) return it->second;
    std::string env = "PE_";
    for (char c : k) env += (c == '-') ? '_' : char(std::toupper(c));
    if (const char* e = std::getenv(env.c_str())) return e;
    return def;
  }
  long long geti(const std::string& k, long long def) const { return std::atoll(get(k, std::to_string(def)).c_str()); }
  double getd(const std::string& k, double def) const {
    const std::string v = get(k, "");
    return v.empty() ? def : std::atof(v.c_str());
  }
  bool flag(const std::string& k) const {
    const std::string v = get(k, "");
    return !v.empty() && v != "0" && v != "false";
  }
  const std::vector<std::string>& positional() const { return pos_; }

 private:
  static bool is_bool_flag(const std::string& k) {
    static const char* b[] = {"json", "legacy", "verbose", "no-graph", "graph", "timing", "no-tol", "help", "history", "quiet"};
    for (auto* s : b)
      if (k == s) return true;
    return false;
  }
  std::map<std::string, std::string> kv_;
  std::vector<std::string> pos_;
};

}  // namespace pe
