#include "aqz_copy.hh"

#include <pthread.h>
#include <sched.h>

#include <cctype>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>

namespace aqz {

std::vector<int>
numa_cpus_for_pci(const char* bus_id, int* node_out)
{
    std::vector<int> cpus;
    if (node_out)
        *node_out = -1;
    if (!bus_id || !*bus_id)
        return cpus;
    std::string id(bus_id);
    for (auto& ch : id)
        ch = char(std::tolower(static_cast<unsigned char>(ch)));
    int node = -1;
    {
        std::ifstream f("/sys/bus/pci/devices/" + id + "/numa_node");
        if (!(f >> node) || node < 0)
            return cpus;
    }
    if (node_out)
        *node_out = node;
    std::ifstream f("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist");
    std::string list;
    if (!std::getline(f, list))
        return cpus;
    cpu_set_t allowed;
    CPU_ZERO(&allowed);
    if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0)
        return cpus;
    std::stringstream ss(list);
    std::string part;
    while (std::getline(ss, part, ',')) {
        int a = -1, b = -1;
        if (std::sscanf(part.c_str(), "%d-%d", &a, &b) == 2) {
        } else if (std::sscanf(part.c_str(), "%d", &a) == 1) {
            b = a;
        } else {
            continue;
        }
        for (int c = a; c <= b && c < CPU_SETSIZE; ++c)
            if (c >= 0 && CPU_ISSET(c, &allowed))
                cpus.push_back(c);
    }
    return cpus;
}

void
pin_current_thread(const std::vector<int>& cpus)
{
    if (cpus.empty())
        return;
    cpu_set_t set;
    CPU_ZERO(&set);
    for (int c : cpus)
        CPU_SET(c, &set);
    (void)pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
}

CopyPool::CopyPool(unsigned workers, std::vector<int> cpus)
{
    for (unsigned i = 0; i < workers; ++i)
        threads_.emplace_back([this, i, cpus] {
            pin_current_thread(cpus);
            run(i);
        });
}

CopyPool::~CopyPool()
{
    {
        std::lock_guard<std::mutex> g(mu_);
        stop_ = true;
    }
    go_.notify_all();
    for (auto& t : threads_)
        t.join();
}

void
CopyPool::piece(size_t i)
{
    const size_t per = (n_ + pieces_ - 1) / pieces_;
    const size_t lo = i * per;
    if (lo >= n_)
        return;
    const size_t len = lo + per > n_ ? n_ - lo : per;
    std::memcpy(dst_ + lo, src_ + lo, len);
}

void
CopyPool::run(unsigned id)
{
    uint64_t seen = 0;
    for (;;) {
        {
            std::unique_lock<std::mutex> lk(mu_);
            go_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_)
                return;
            seen = gen_;
        }
        piece(id + 1); // piece 0 is the caller's
        {
            std::lock_guard<std::mutex> g(mu_);
            if (--pending_ == 0)
                done_.notify_one();
        }
    }
}

void
CopyPool::copy(void* dst, const void* src, size_t n)
{
    constexpr size_t kMinPiece = size_t(4) << 20;
    if (threads_.empty() || n < 2 * kMinPiece) {
        std::memcpy(dst, src, n);
        return;
    }
    {
        std::lock_guard<std::mutex> g(mu_);
        dst_ = static_cast<uint8_t*>(dst);
        src_ = static_cast<const uint8_t*>(src);
        n_ = n;
        pieces_ = threads_.size() + 1;
        pending_ = unsigned(threads_.size());
        ++gen_;
    }
    go_.notify_all();
    piece(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return pending_ == 0; });
}

} // namespace aqz
