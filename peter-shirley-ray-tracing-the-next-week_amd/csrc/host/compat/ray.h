// compat/ray.h — reference header name; see rtnw_compat.h
#pragma once
#include "rtnw_compat.h"
