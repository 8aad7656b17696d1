// praos_kernels.h -- shared definitions between the kernels and the C ABI.
#pragma once
#include "praos_hip.h"
