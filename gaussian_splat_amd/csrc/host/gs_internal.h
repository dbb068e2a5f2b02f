// gs_internal.h — library-internal helpers shared by the host translation
// units of libgsplat.so (not part of the C-ABI).
#pragma once

#include <string>

// Sets gs_last_error() of the calling thread (renderer.cpp).
void gs_set_last_error(const std::string& msg);
