#include "aqz_copy.hh"

#include <cstring>

namespace aqz {

CopyPool::CopyPool(unsigned workers)
{
    for (unsigned i = 0; i < workers; ++i)
        threads_.emplace_back([this, i] { run(i); });
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
