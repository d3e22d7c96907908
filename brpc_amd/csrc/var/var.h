// Umbrella header for the metrics layer (role of bvar/bvar.h).
#pragma once

#include "var/gflag.h"
#include "var/lock_timer.h"
#include "var/multi_dimension.h"
#include "var/percentile.h"
#include "var/recorder.h"
#include "var/reducer.h"
#include "var/variable.h"
#include "var/window.h"
