// Timer-driven periodic tasks (reference src/brpc/periodic_task.h:33-40):
// OnTriggeringTask runs in a fiber at each deadline; it returns false to
// stop, or true and sets the next deadline. OnDestroyingTask is called once
// the task stops (or the manager is told to stop everything at exit).
#pragma once

#include <ctime>

namespace mrpc {

class PeriodicTask {
public:
    virtual ~PeriodicTask() {}
    // Return true to run again at *next_abstime.
    virtual bool OnTriggeringTask(timespec* next_abstime) = 0;
    virtual void OnDestroyingTask() = 0;
};

class PeriodicTaskManager {
public:
    // Run task at abstime (and again while it asks to).
    static void StartTaskAt(PeriodicTask* task, const timespec& abstime);
};

}  // namespace mrpc
