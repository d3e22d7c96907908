// Umbrella header for the metrics layer (role of bvar/bvar.h).
#pragma once

#include "var/percentile.h"
#include "var/recorder.h"
#include "var/reducer.h"
#include "var/variable.h"
#include "var/window.h"
