#pragma once
#include "octomap.h"
