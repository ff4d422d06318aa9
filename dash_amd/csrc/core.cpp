// dash_amd native core implementation (see core.h).
#include "core.h"

#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>

#include <wmmintrin.h>

namespace dash {

std::vector<int> first_primes(int k) {
    DASH_CHECK(k > 0, "number of primes must be positive");
    std::vector<int> out;
    for (int c = 2; static_cast<int>(out.size()) < k; ++c) {
        bool prime = true;
        for (int d : out) {
            if (d * d > c) break;
            if (c % d == 0) {
                prime = false;
                break;
            }
        }
        if (prime) out.push_back(c);
    }
    return out;
}

// ---------------------------------------------------------------------------
namespace {
constexpr int kMaxMod = 4096;
struct ModTable {
    ModInfo info[kMaxMod];
    ModTable() {
        for (int p = 2; p < kMaxMod; ++p) {
            ModInfo& m = info[p];
            m.p = p;
            m.n = nr_comps(p);
            m.pow2 = (p & (p - 1)) == 0;
            if (m.pow2) {
                int b = 0;
                while ((1 << b) < p) ++b;
                m.bits = b;
            }
            u64 pc = p;
            int c = 1;
            while (pc * static_cast<u64>(p) < (1ull << 32)) {
                pc *= p;
                ++c;
            }
            m.chunk = c;
            m.pchunk = pc;
            m.prg_m = prg_digits(p);
        }
    }
};
const ModTable& mod_table() {
    static ModTable t;
    return t;
}
}  // namespace

void* big_alloc(size_t bytes, bool* zeroed) {
    if (bytes >= kBigAlloc) {
        void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p == MAP_FAILED) throw std::bad_alloc();
        madvise(p, bytes, MADV_HUGEPAGE);
        if (zeroed) *zeroed = true;
        return p;
    }
    void* p = std::aligned_alloc(64, (bytes + 63) & ~size_t(63));
    if (!p) throw std::bad_alloc();
    if (zeroed) *zeroed = false;
    return p;
}

void big_free(void* p, size_t bytes) {
    if (!p) return;
    if (bytes >= kBigAlloc)
        munmap(p, bytes);
    else
        std::free(p);
}

const ModInfo& mod_info(int p) {
    DASH_CHECK(p >= 2 && p < kMaxMod, "modulus out of supported range [2, 4096)");
    return mod_table().info[p];
}

// ---------------------------------------------------------------------------
// AES-128 key schedule with AES-NI
namespace {
inline __m128i expand_step(__m128i key, __m128i gen) {
    gen = _mm_shuffle_epi32(gen, 0xff);
    key = _mm_xor_si128(key, _mm_slli_si128(key, 4));
    key = _mm_xor_si128(key, _mm_slli_si128(key, 4));
    key = _mm_xor_si128(key, _mm_slli_si128(key, 4));
    return _mm_xor_si128(key, gen);
}
}  // namespace

void aes_expand(const uint8_t key[16], AesKey& out) {
    __m128i k = _mm_loadu_si128(reinterpret_cast<const __m128i*>(key));
    out.rk[0] = k;
    k = expand_step(k, _mm_aeskeygenassist_si128(k, 0x01)); out.rk[1] = k;
    k = expand_step(k, _mm_aeskeygenassist_si128(k, 0x02)); out.rk[2] = k;
    k = expand_step(k, _mm_aeskeygenassist_si128(k, 0x04)); out.rk[3] = k;
    k = expand_step(k, _mm_aeskeygenassist_si128(k, 0x08)); out.rk[4] = k;
    k = expand_step(k, _mm_aeskeygenassist_si128(k, 0x10)); out.rk[5] = k;
    k = expand_step(k, _mm_aeskeygenassist_si128(k, 0x20)); out.rk[6] = k;
    k = expand_step(k, _mm_aeskeygenassist_si128(k, 0x40)); out.rk[7] = k;
    k = expand_step(k, _mm_aeskeygenassist_si128(k, 0x80)); out.rk[8] = k;
    k = expand_step(k, _mm_aeskeygenassist_si128(k, 0x1b)); out.rk[9] = k;
    k = expand_step(k, _mm_aeskeygenassist_si128(k, 0x36)); out.rk[10] = k;
}

void aes_round_key_bytes(const AesKey& k, uint8_t out[176]) {
    for (int r = 0; r < 11; ++r) _mm_storeu_si128(reinterpret_cast<__m128i*>(out + 16 * r), k.rk[r]);
}

const AesKey& fixed_key() {
    static AesKey k = [] {
        AesKey kk;
        uint8_t key[16];
        for (int i = 0; i < 16; ++i) key[i] = static_cast<uint8_t>(i);
        aes_expand(key, kk);
        return kk;
    }();
    return k;
}

void hash_batch(const u128* in, u128* out, size_t n) {
    const AesKey& k = fixed_key();
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        __m128i x[8];
        for (int j = 0; j < 8; ++j) x[j] = _mm_xor_si128(u128_to_m(in[i + j]), k.rk[0]);
        for (int r = 1; r < 10; ++r)
            for (int j = 0; j < 8; ++j) x[j] = _mm_aesenc_si128(x[j], k.rk[r]);
        for (int j = 0; j < 8; ++j) out[i + j] = m_to_u128(_mm_aesenclast_si128(x[j], k.rk[10]));
    }
    for (; i < n; ++i) out[i] = hash(in[i]);
}

// ---------------------------------------------------------------------------
// Thread pool
namespace {
class Pool {
   public:
    explicit Pool(int n) : nthreads_(n) {
        const int base = std::max(0, sched_getcpu());  // the caller (thread 0) keeps its CPU
        for (int i = 1; i < n; ++i)
            workers_.emplace_back([this, i, base] {
                spread(base + i);
                loop(i);
            });
    }
    // Move worker i onto the i-th allowed CPU once, then restore the full mask.
    // Some VM guests (observed: firecracker microVMs) never load-balance new
    // threads away from their parent's CPU, so an unpinned pool ran all its
    // workers on one core. The mask is restored, so the OS may still migrate.
    static void spread(int i) {
        cpu_set_t all;
        CPU_ZERO(&all);
        if (sched_getaffinity(0, sizeof(all), &all) != 0) return;
        const int cnt = CPU_COUNT(&all);
        if (cnt <= 1) return;
        int want = i % cnt, seen = 0, cpu = -1;  // i counts allowed CPUs from the caller's
        for (int c = 0; c < CPU_SETSIZE; ++c)
            if (CPU_ISSET(c, &all) && seen++ == want) {
                cpu = c;
                break;
            }
        if (cpu < 0) return;
        cpu_set_t one;
        CPU_ZERO(&one);
        CPU_SET(cpu, &one);
        if (pthread_setaffinity_np(pthread_self(), sizeof(one), &one) != 0) return;
        sched_yield();
        pthread_setaffinity_np(pthread_self(), sizeof(all), &all);
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
            ++gen_;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }
    int size() const { return nthreads_; }
    // Runs job(tid) on threads 0..use-1 (the caller is thread 0).
    void run(int use, const std::function<void(int)>& job) {
        std::unique_lock<std::mutex> run_lk(run_mu_);
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &job;
            use_ = use;
            pending_ = use - 1;
            ++gen_;
        }
        cv_.notify_all();
        std::exception_ptr err;
        try {
            job(0);
        } catch (...) {
            err = std::current_exception();
        }
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [this] { return pending_ == 0; });
        job_ = nullptr;
        if (!err && worker_err_) err = worker_err_;
        worker_err_ = nullptr;
        lk.unlock();
        if (err) std::rethrow_exception(err);
    }

   private:
    void loop(int tid) {
        u64 seen = 0;
        for (;;) {
            const std::function<void(int)>* job;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                if (tid >= use_) continue;
                job = job_;
            }
            std::exception_ptr err;
            try {
                (*job)(tid);
            } catch (...) {
                err = std::current_exception();
            }
            {
                std::lock_guard<std::mutex> lk(mu_);
                if (err && !worker_err_) worker_err_ = err;
                if (--pending_ == 0) done_cv_.notify_all();
            }
        }
    }
    int nthreads_;
    std::vector<std::thread> workers_;
    std::mutex mu_, run_mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(int)>* job_ = nullptr;
    int use_ = 0;
    int pending_ = 0;
    u64 gen_ = 0;
    bool stop_ = false;
    std::exception_ptr worker_err_;
};

std::atomic<int> g_default_threads{0};

int hw_threads() {
    unsigned h = std::thread::hardware_concurrency();
    return h == 0 ? 1 : static_cast<int>(h);
}

Pool& pool() {
    static Pool p(std::max(1, std::min(hw_threads(), 64)));
    return p;
}
thread_local bool t_in_pool = false;
}  // namespace

int default_threads() {
    int n = g_default_threads.load();
    if (n <= 0) {
        const char* env = std::getenv("DASH_NUM_THREADS");
        n = env ? std::atoi(env) : std::min(hw_threads(), 16);
        if (n <= 0) n = 1;
    }
    return n;
}
void set_default_threads(int n) { g_default_threads.store(n); }

void parallel_for(i64 n, const std::function<void(i64, i64)>& body, int nthreads) {
    if (n <= 0) return;
    int nt = nthreads > 0 ? nthreads : default_threads();
    nt = std::min<i64>(nt, n);
    nt = std::min(nt, pool().size());
    if (nt <= 1 || t_in_pool) {
        body(0, n);
        return;
    }
    i64 chunk = (n + nt - 1) / nt;
    std::function<void(int)> job = [&](int tid) {
        t_in_pool = true;
        i64 b = tid * chunk, e = std::min(n, b + chunk);
        if (b < e) body(b, e);
        t_in_pool = false;
    };
    pool().run(nt, job);
}

}  // namespace dash
