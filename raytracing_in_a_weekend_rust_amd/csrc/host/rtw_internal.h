// rtw_internal.h -- shared between the host mirror (rtw_host.cpp) and the device
// half of the C ABI (rtw_render.hip). Not part of the public ABI.
#pragma once

#include <string>

namespace rtw {
void set_error(const std::string &m);
const char *last_error();
}  // namespace rtw
