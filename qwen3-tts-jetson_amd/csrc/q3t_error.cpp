#include "q3t_common.h"
namespace q3t {
static thread_local std::string g_err;
void set_error(const std::string &m) { g_err = m; }
const std::string &last_error() { return g_err; }
}
