// TEST stub: opencv2/opencv.hpp -> the declaration-only core (see core/core.hpp)
#pragma once
#include "core/core.hpp"
