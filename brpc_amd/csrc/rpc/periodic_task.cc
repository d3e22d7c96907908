#include "rpc/periodic_task.h"

#include "base/logging.h"
#include "fiber/fiber.h"

namespace mrpc {

namespace {

void* RunPeriodicTask(void* arg);

void OnTimer(void* arg) {
    // Timer callbacks must be short: hand the task to a fiber.
    fiber::fiber_t th;
    if (fiber::start_background(&th, &fiber::ATTR_NORMAL, RunPeriodicTask, arg) != 0) RunPeriodicTask(arg);
}

void* RunPeriodicTask(void* arg) {
    PeriodicTask* task = static_cast<PeriodicTask*>(arg);
    timespec next = {0, 0};
    if (!task->OnTriggeringTask(&next)) {
        task->OnDestroyingTask();
        return nullptr;
    }
    PeriodicTaskManager::StartTaskAt(task, next);
    return nullptr;
}

}  // namespace

void PeriodicTaskManager::StartTaskAt(PeriodicTask* task, const timespec& abstime) {
    if (!task) return;
    fiber::init_runtime();
    fiber::TimerId id;
    if (fiber::timer_add(&id, abstime, OnTimer, task) != 0) {
        LOG(ERROR) << "Fail to schedule a periodic task; running it now";
        OnTimer(task);
    }
}

}  // namespace mrpc
