#pragma once

#include "fiber/fiber.h"

namespace mrpc {
namespace fiber {

struct KeyTable;
// Called by the scheduler when a fiber ends: runs destructors, or returns the
// table to `pool` (keeping data) when the fiber was started with one.
void return_keytable(KeyTablePool* pool, KeyTable* kt);
KeyTable* borrow_keytable(KeyTablePool* pool);

}  // namespace fiber
}  // namespace mrpc
