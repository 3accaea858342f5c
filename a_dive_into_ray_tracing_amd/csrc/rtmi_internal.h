// rtmi_internal.h — shared between the host (rtmi_host.cpp) and device
// (rtmi_device.hip) halves of librtmi.so.  Not installed.
#pragma once

#include "../../include/rtmi.h"

#define RTMI_EXPORT extern "C" __attribute__((visibility("default")))

namespace rtmi {
int set_error(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
void clear_error();
}  // namespace rtmi
