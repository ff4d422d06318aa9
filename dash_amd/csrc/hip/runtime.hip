// HIP evaluator runtime: uploads a batch of B garbled models (same circuit,
// independent garblings) into an HBM arena and evaluates them together, one
// kernel launch per gadget phase over (GC x residue x element). All launches
// go to one stream (no per-layer device synchronisation, unlike the
// reference's cudaDeviceSynchronize after every layer), so the whole forward
// can be captured into a hipGraph.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <atomic>
#include <cstring>
#include <tuple>
#include <chrono>
#include <map>
#include <mutex>
#include <functional>
#include <thread>

#include "../layers.h"
#include "host_util.h"
#include "launch.h"
#include "fetch.h"

#include <rocprofiler-sdk-roctx/roctx.h>

namespace py = pybind11;

namespace dash {
using namespace dev;

using namespace hostutil;

// ---------------------------------------------------------------------------
// Garbler side of the same-node device transport: another process's evaluator table arenas opened through their
// IPC handles (HipEvaluator::ipc_export), handed to the GPU garbler as slot sinks. The garbler's kernels write
// the tables straight into the evaluator's HBM (its own device, or a peer over xGMI); only the skeleton of each
// model (constants, shapes) then travels over the channel.
class IpcTables {
   public:
    IpcTables(int device, const std::vector<std::tuple<size_t, std::string, size_t, std::string>>& handles, int B)
        : dev_(device), B_(B), alive_(std::make_shared<std::atomic<bool>>(true)) {
        DASH_CHECK(B >= 1, "IpcTables: batch must be >= 1");
        bind_device(dev_, nullptr, "IpcTables");
        for (const auto& h : handles) {
            const std::string& hb = std::get<3>(h);
            DASH_CHECK(hb.size() == sizeof(hipIpcMemHandle_t), "IpcTables: bad IPC handle size");
            hipIpcMemHandle_t mh;
            std::memcpy(&mh, hb.data(), sizeof(mh));
            void* p = nullptr;
            HIPCHECK(hipIpcOpenMemHandle(&p, mh, hipIpcMemLazyEnablePeerAccess));
            opened_.push_back(p);
            map_[{std::get<0>(h), std::get<1>(h)}] = {static_cast<uint8_t*>(p), std::get<2>(h)};
        }
    }
    ~IpcTables() {
        alive_->store(false);
        (void)hipSetDevice(dev_);
        for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
        (void)hipGetLastError();  // teardown errors are ignored: do not leave them for a later HIPCHECK
    }
    int tables() const { return static_cast<int>(map_.size()); }
    std::shared_ptr<TableSink> sink(int b) const {
        DASH_CHECK(b >= 0 && b < B_, "IpcTables: batch slot out of range");
        auto map = map_;
        const int dev = dev_;
        auto alive = alive_;
        auto s = std::make_shared<TableSink>();
        s->dest = [map, b, dev, alive](size_t layer, const std::string& name, size_t nbytes) -> std::shared_ptr<Array::Device> {
            auto it = map.find({layer, name});
            if (it == map.end() || it->second.second != nbytes) return nullptr;
            auto d = std::make_shared<Array::Device>();
            d->p = std::shared_ptr<void>(it->second.first + nbytes * b, [](void*) {});  // the evaluator owns it
            d->device = dev;
            d->external = true;
            d->fetch = [dev, alive](void* h, const void* dv, size_t n) {
                if (!alive->load())
                    throw std::runtime_error("dash: tables live in a closed IPC mapping of the evaluator's slots");
                HIPCHECK(hipSetDevice(dev));
                HIPCHECK(hipMemcpy(h, dv, n, hipMemcpyDeviceToHost));
            };
            return d;
        };
        return s;
    }

   private:
    int dev_, B_;
    std::shared_ptr<std::atomic<bool>> alive_;
    std::vector<void*> opened_;
    std::map<std::pair<size_t, std::string>, std::pair<uint8_t*, size_t>> map_;
};

// ---------------------------------------------------------------------------
class HipEvaluator {
   public:
    HipEvaluator(std::shared_ptr<GarbledModel> tmpl, int B, int device, bool use_mfma, bool stream_tables = false)
        : tmpl_(std::move(tmpl)), mfma_(use_mfma), stream_(stream_tables) {
        DASH_CHECK(tmpl_ && B >= 1, "HipEvaluator needs a template model and B >= 1");
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
            throw std::runtime_error("dash: no HIP device available for HipEvaluator");
        dev_ = device;
        HIPCHECK(hipSetDevice(dev_));
        B_ = B;
        crt_ = tmpl_->h.crt;
        k_ = static_cast<int>(crt_.size());
        for (int p : crt_)
            DASH_CHECK(p <= kActMaxModulus, "HIP evaluator: CRT modulus " + std::to_string(p) +
                                                " > 255 (activations are stored as bytes); use the host evaluator");
        DASH_CHECK(k_ <= kMaxRes, "too many CRT residues for the GPU path");
        loaded_.assign(B_, 0);
        build();
        // Keep only what load() checks: holding the template model would pin
        // its garbled tables (10 GB per MiniONN GC, device-resident when the
        // GPU garbler made them) for the evaluator's lifetime.
        tmpl_h_ = tmpl_->h;
        tmpl_nlayers_ = tmpl_->layers.size();
        tmpl_.reset();
    }
    // Upload garbled model `m` (same circuit as the template) into batch slot b.
    void load(int b, const GarbledModel& m) {
        DASH_CHECK(b >= 0 && b < B_, "batch slot out of range");
        // one load at a time: the per-GC constants go through ONE pinned staging block, device block and load
        // stream shared by all slots (the serving engine's refill workers load different slots of one evaluator
        // concurrently; unserialized, one slot's constants could land in another's)
        std::lock_guard<std::mutex> load_guard(load_mu_);
        DASH_CHECK(m.h.crt == tmpl_h_.crt && m.h.mrs == tmpl_h_.mrs && m.layers.size() == tmpl_nlayers_ &&
                       m.h.in_dims == tmpl_h_.in_dims && m.h.hardened == tmpl_h_.hardened,
                   "model does not garble the evaluator's circuit (or uses another encoding)");
        bind_device(dev_, load_st_, "HipEvaluator.load");
        if (!load_st_) HIPCHECK(hipStreamCreateWithFlags(&load_st_, hipStreamNonBlocking));
        // per-GC small constants (bias labels, zero / shift labels, ...): filled into one pinned staging block,
        // one H2D copy and one scatter kernel to their slot-b destinations, instead of ~100 small copies
        if (!small_.empty()) {
            for (const auto& c : small_) c.fill(m, small_h_ + c.off);
            HIPCHECK(hipMemcpyAsync(small_d_, small_h_, small_bytes_, hipMemcpyHostToDevice, load_st_));
            launch_scatter(small_desc_, static_cast<int>(small_.size()), small_d_, b, load_st_);
        }
        // tables (a GC garbled into this slot through sink() needs none of these copies)
        for (auto& f : loaders_) f(b, m);
        // evaluation and garbling streams are non-blocking: this waits for this load only
        HIPCHECK(hipStreamSynchronize(load_st_));
        loaded_[b] = 1;
    }
    // Zero-copy offline phase (GarbleOptions::sink): slot b's table arenas as GPU-garbler destinations.
    // A model garbled with this sink already has its tables in slot b, and load(b, m) skips their copies.
    std::shared_ptr<TableSink> sink(int b) const {
        DASH_CHECK(b >= 0 && b < B_, "batch slot out of range");
        auto arena = arena_;
        const int dev = dev_;
        auto alive = alive_;
        auto s = std::make_shared<TableSink>();
        s->dest = [arena, b, dev, alive](size_t layer, const std::string& name, size_t nbytes) -> std::shared_ptr<Array::Device> {
            auto it = arena.find({layer, name});
            if (it == arena.end() || it->second.second != nbytes) return nullptr;
            auto d = std::make_shared<Array::Device>();
            d->p = std::shared_ptr<void>(it->second.first + nbytes * b, [](void*) {});  // the evaluator owns it
            d->device = dev;
            d->external = true;
            // the arena belongs to the evaluator: a model that outlives it must not read freed HBM
            d->fetch = [dev, alive](void* h, const void* dv, size_t n) {
                if (!alive->load())
                    throw std::runtime_error("dash: garbled tables live in a destroyed HipEvaluator's slot (sink); "
                                             "the model is no longer readable");
                HIPCHECK(hipSetDevice(dev));
                HIPCHECK(hipMemcpy(h, dv, n, hipMemcpyDeviceToHost));
            };
            return d;
        };
        return s;
    }
    // Same-node device transport (net/protocol.py, transport "ipc"): an IPC handle per table arena, so a
    // garbler process can garble straight into this evaluator's slots (IpcTables). Entries: (layer, table,
    // bytes per slot, handle bytes).
    std::vector<std::tuple<size_t, std::string, size_t, std::string>> ipc_export() const {
        bind_device(dev_, nullptr, "HipEvaluator.ipc_export");
        DASH_CHECK(!stream_, "ipc export needs HBM-resident tables (stream_tables=False)");
        std::vector<std::tuple<size_t, std::string, size_t, std::string>> out;
        for (const auto& kv : arena_) {
            hipIpcMemHandle_t h;
            HIPCHECK(hipIpcGetMemHandle(&h, kv.second.first));
            out.emplace_back(kv.first.first, kv.first.second, kv.second.second,
                             std::string(reinterpret_cast<const char*>(&h), sizeof(h)));
        }
        return out;
    }
    ~HipEvaluator() {
        alive_->store(false);  // orphans every sink-backed model array (fetch raises instead of reading freed HBM)
        if (copy_st_) (void)hipStreamSynchronize(copy_st_);
        for (auto e : ready_) (void)hipEventDestroy(e);
        for (auto e : done_) (void)hipEventDestroy(e);
        if (run_end_) (void)hipEventDestroy(run_end_);
        if (copy_st_) (void)hipStreamDestroy(copy_st_);
        if (load_st_) (void)hipStreamDestroy(load_st_);
        if (gexec_) (void)hipGraphExecDestroy(gexec_);
        for (void* p : allocs_) (void)hipFree(p);
        for (void* p : host_allocs_) (void)hipHostFree(p);
        (void)hipGetLastError();  // teardown errors are ignored: do not leave them for a later HIPCHECK
    }

    int batch() const { return B_; }
    bool streams_tables() const { return stream_; }
    size_t device_bytes() const { return dev_bytes_; }
    size_t table_bytes() const { return table_bytes_; }

    void set_inputs(const std::vector<CrtLabels>& in, hipStream_t st) {
        DASH_CHECK(static_cast<int>(in.size()) == B_, "need one input per garbled model in the batch");
        for (int j = 0; j < k_; ++j) {
            const int n = nr_comps(crt_[j]);
            int16_t* stg = in_stage_[j];
            for (int b = 0; b < B_; ++b) {
                const Labels& L = in[b][j];
                DASH_CHECK(L.p == crt_[j] && L.N == N0_, "input label shape mismatch");
                for (i64 e = 0; e < N0_; ++e)
                    for (int c = 0; c < n; ++c) stg[(static_cast<i64>(b) * n + c) * N0_ + e] = L.c[e * n + c];
            }
        }
        upload_inputs(st);
    }

    // pinned staging slots for GC b (one component-major block per residue)
    std::vector<int16_t*> input_slot(int b) const {
        DASH_CHECK(b >= 0 && b < B_, "batch slot out of range");
        std::vector<int16_t*> v;
        for (int j = 0; j < k_; ++j) v.push_back(in_stage_[j] + static_cast<i64>(b) * nr_comps(crt_[j]) * N0_);
        return v;
    }
    i64 input_size() const { return N0_; }
    int device() const { return dev_; }
    const std::vector<int>& crt() const { return crt_; }
    // slot b's device input activations of residue j, [n_j][N0] bytes: the target of the garbler's device encoder
    act_t* input_act(int b, int j) const {
        DASH_CHECK(b >= 0 && b < B_ && j >= 0 && j < k_, "input slot out of range");
        return bufs_[0].p[j] + static_cast<i64>(b) * nr_comps(crt_[j]) * N0_;
    }
    // compressed staging (online message #1 in wire form): [B][k][N0] u128
    u128* input_slot_compressed(int b) {
        DASH_CHECK(b >= 0 && b < B_, "batch slot out of range");
        if (!in_comp_stage_) {
            bind_device(dev_, nullptr, "HipEvaluator.input_slot_compressed");
            const size_t bytes = sizeof(u128) * B_ * k_ * N0_;
            HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&in_comp_stage_), bytes));
            host_allocs_.push_back(in_comp_stage_);
            HIPCHECK(hipMalloc(reinterpret_cast<void**>(&in_comp_dev_), bytes));
            allocs_.push_back(in_comp_dev_);
            dev_bytes_ += bytes;
        }
        return in_comp_stage_ + static_cast<i64>(b) * k_ * N0_;
    }
    void upload_inputs_compressed(hipStream_t st) {
        bind_device(dev_, st, "HipEvaluator.upload_inputs_compressed");
        DASH_CHECK(in_comp_stage_ != nullptr, "no compressed inputs staged");
        HIPCHECK(hipMemcpyAsync(in_comp_dev_, in_comp_stage_, sizeof(u128) * B_ * k_ * N0_, hipMemcpyHostToDevice, st));
        launch_unpack(in_comp_dev_, k_, bufs_[0], crt_info(crt_), mc_, N0_, B_, st);
    }
    // output labels of slot b, compressed on the host: [k][Nout]
    std::vector<u128> outputs_compressed(int b) const {
        std::vector<u128> r(static_cast<size_t>(k_) * Nout_);
        for (int j = 0; j < k_; ++j) {
            const ModInfo& mi = mod_info(out_mod_[j]);
            comp_t buf[128];
            for (i64 e = 0; e < Nout_; ++e) {
                for (int c = 0; c < mi.n; ++c) buf[c] = out_stage_[j][(static_cast<i64>(b) * mi.n + c) * Nout_ + e];
                r[static_cast<size_t>(j) * Nout_ + e] = compress(buf, mi);
            }
        }
        return r;
    }
    // every residue's output labels -> out_stage_: one k_fetch_res launch into the mapped pinned buffers for small
    // outputs (one launch instead of k copy-engine transfers), copies otherwise or with DASH_FETCH_KERNEL=0 (A/B)
    void stage_outputs(hipStream_t st) {
        static const bool kern = [] {
            const char* e = std::getenv("DASH_FETCH_KERNEL");
            return !(e && e[0] == '0');
        }();
        FetchRes f{};
        f.k = k_;
        int64_t total = 0;
        for (int j = 0; j < k_; ++j) {
            f.in[j] = final_.p[j];
            f.out[j] = out_stage_dev_[j];
            f.bytes[j] = static_cast<int64_t>(sizeof(act_t)) * B_ * nr_comps(out_mod_[j]) * Nout_;
            total += f.bytes[j];
        }
        if (kern && total <= (4 << 20) && out_stage_mapped_) {
            launch_fetch_res(f, st);
            HIPCHECK(hipGetLastError());
        } else {
            for (int j = 0; j < k_; ++j)
                HIPCHECK(hipMemcpyAsync(out_stage_[j], final_.p[j], f.bytes[j], hipMemcpyDeviceToHost, st));
        }
        HIPCHECK(hipStreamSynchronize(st));
    }
    void fetch_outputs(hipStream_t st) {
        bind_device(dev_, st, "HipEvaluator.fetch_outputs");
        stage_outputs(st);
    }
    int crt_size() const { return k_; }
    i64 output_size() const { return Nout_; }
    // int16 host staging (the host label format) -> device int16 scratch -> byte activations
    void upload_inputs(hipStream_t st) {
        bind_device(dev_, st, "HipEvaluator.upload_inputs");
        for (int j = 0; j < k_; ++j) {
            const i64 count = static_cast<i64>(B_) * nr_comps(crt_[j]) * N0_;
            if (!in16_dev_[j]) in16_dev_[j] = dalloc<int16_t>(static_cast<size_t>(count));
            HIPCHECK(hipMemcpyAsync(in16_dev_[j], in_stage_[j], sizeof(int16_t) * count, hipMemcpyHostToDevice, st));
            launch_narrow(in16_dev_[j], bufs_[0].p[j], count, st);
        }
    }

    // The op list is static (all device pointers fixed at build time), so
    // after one eager run (lazy one-time allocations) it is captured into a
    // hipGraph and replayed: one launch per evaluation instead of ~200.
    void run(hipStream_t st) {
        bind_device(dev_, st, "HipEvaluator.run");
        for (int b = 0; b < B_; ++b) DASH_CHECK(loaded_[b], "batch slot " + std::to_string(b) + " has no garbled model loaded");
        if (profile_ || !use_graph_ || runs_ == 0 || st == nullptr) {
            // roctx ranges per op (layer / gadget phase) for rocprofv3 --marker-trace (DASH_ROCTX=1)
            static const bool markers = [] {
                const char* e = std::getenv("DASH_ROCTX");
                return e && e[0] == '1';
            }();
            for (size_t i = 0; i < ops_.size(); ++i) {
                if (profile_) HIPCHECK(hipEventRecord(ev_[i], st));
                if (markers) roctxRangePushA(op_names_[i].c_str());
                ops_[i](st);
                if (markers) roctxRangePop();
            }
            if (profile_) HIPCHECK(hipEventRecord(ev_.back(), st));
            HIPCHECK(hipGetLastError());
            ++runs_;
            return;
        }
        if (!gexec_ || gstream_ != st) {
            if (gexec_) HIPCHECK(hipGraphExecDestroy(gexec_));
            gexec_ = nullptr;
            hipGraph_t graph = nullptr;
            HIPCHECK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
            for (auto& op : ops_) op(st);
            HIPCHECK(hipStreamEndCapture(st, &graph));
            HIPCHECK(hipGraphInstantiate(&gexec_, graph, nullptr, nullptr, 0));
            HIPCHECK(hipGraphDestroy(graph));
            gstream_ = st;
        }
        HIPCHECK(hipGraphLaunch(gexec_, st));
        ++runs_;
    }
    void set_graph(bool on) { use_graph_ = on; }

    std::vector<CrtLabels> get_outputs(hipStream_t st) {
        bind_device(dev_, st, "HipEvaluator.get_outputs");
        std::vector<CrtLabels> out(B_);
        stage_outputs(st);
        for (int b = 0; b < B_; ++b)
            for (int j = 0; j < k_; ++j) {
                const int q = out_mod_[j];
                Labels L(q, Nout_);
                const int n = L.n;
                for (i64 e = 0; e < Nout_; ++e)
                    for (int c = 0; c < n; ++c) L.c[e * n + c] = out_stage_[j][(static_cast<i64>(b) * n + c) * Nout_ + e];
                out[b].push_back(std::move(L));
            }
        return out;
    }

    void set_profile(bool on) {
        profile_ = on;
        if (on && ev_.empty()) {
            bind_device(dev_, nullptr, "HipEvaluator.set_profile");
            ev_.resize(ops_.size() + 1);
            for (auto& e : ev_) HIPCHECK(hipEventCreate(&e));
        }
    }
    std::vector<std::pair<std::string, double>> op_times() const {
        std::vector<std::pair<std::string, double>> r;
        if (!profile_) return r;
        for (size_t i = 0; i < ops_.size(); ++i) {
            float ms = 0;
            (void)hipEventElapsedTime(&ms, ev_[i], ev_[i + 1]);
            r.emplace_back(op_names_[i], ms);
        }
        return r;
    }

   private:
    std::shared_ptr<std::atomic<bool>> alive_ = std::make_shared<std::atomic<bool>>(true);
    // ------------------------------------------------------------ helpers
    template <typename T>
    T* dalloc(size_t count) {
        void* p = nullptr;
        size_t bytes = std::max<size_t>(count * sizeof(T), 64);
        HIPCHECK(hipMalloc(&p, bytes));
        allocs_.push_back(p);
        dev_bytes_ += bytes;
        return static_cast<T*>(p);
    }
    template <typename T>
    T* upload(const T* host, size_t count) {
        T* d = dalloc<T>(count);
        HIPCHECK(hipMemcpy(d, host, count * sizeof(T), hipMemcpyHostToDevice));
        return d;
    }
    // a model array into device memory: device-to-device (or peer) when the GPU
    // garbler left it in HBM and nobody has fetched (and possibly edited) a host copy
    static void copy_in(uint8_t* dst, const Array& a, hipStream_t st) {
        if (a.in_slot) return;  // skeleton model: the garbler wrote these bytes into this slot (IPC sink)
        if (a.device_resident() && a.device_ptr() == dst) return;  // garbled straight into this slot (sink)
        if (a.device_resident() && !a.dev->host)
            HIPCHECK(hipMemcpyAsync(dst, a.device_ptr(), a.nbytes, hipMemcpyDefault, st));
        else  // pageable host source: staged before the call returns
            HIPCHECK(hipMemcpyAsync(dst, a.ptr<uint8_t>(), a.nbytes, hipMemcpyHostToDevice, st));
    }
    // a per-GC small constant of `bytes` at dst0 + b * stride for slot b, filled on the host by `fill`
    void add_small(uint8_t* dst0, size_t stride, size_t bytes, std::function<void(const GarbledModel&, uint8_t*)> fill) {
        SmallLoad c;
        c.off = small_bytes_;
        c.dst0 = dst0;
        c.stride = stride;
        c.bytes = bytes;
        c.fill = std::move(fill);
        small_bytes_ += (bytes + 15) / 16 * 16;
        small_.push_back(std::move(c));
    }
    // after build(): staging buffers and the device descriptor table of the small constants
    void finish_small() {
        if (small_.empty()) return;
        HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&small_h_), small_bytes_));
        host_allocs_.push_back(small_h_);
        small_d_ = dalloc<uint8_t>(small_bytes_);
        std::vector<ScatterDesc> d;
        for (const auto& c : small_) d.push_back(ScatterDesc{c.off, c.dst0, c.stride, c.bytes});
        small_desc_ = upload(d.data(), d.size());
    }
    // one device buffer holding array `name` of layer li of every GC slot
    const u128* upload_tables(size_t li, const std::string& name) {
        const size_t nb = tmpl_->layers[li].arr(name).nbytes;
        if (stream_) return stream_table(li, name, nb);
        uint8_t* d = dalloc<uint8_t>(nb * B_);
        arena_[{li, name}] = {d, nb};
        loaders_.push_back([this, d, nb, li, name](int b, const GarbledModel& m) {
            const Array& a = m.layers[li].arr(name);
            DASH_CHECK(a.nbytes == nb, "table size mismatch across batch");
            copy_in(d + nb * b, a, load_st_);
        });
        table_bytes_ += nb * B_;
        return reinterpret_cast<const u128*>(d);
    }
    // Streamed tables (stream_tables): every GC's copy of the array lives in pinned host memory; the layer's
    // tables of all B slots are copied into one of three rotating HBM windows on a copy stream one layer
    // ahead of their use (stage_layer), so the device holds at most three layers of tables. For models (or
    // batches) whose tables exceed the HBM pool; the reference uploads every table at load (sign_gadget.h
    // cuda_move, 708-734). Three windows because a joint rescale's op runs in the next layer, reading its
    // own layer's tables: layer x's window is reused by layer x + 3 only after layer x + 1 has finished.
    const u128* stream_table(size_t li, const std::string& name, size_t nb) {
        const size_t span = (nb * B_ + 255) / 256 * 256;
        DASH_CHECK(woff_[li] + span <= win_bytes_, "streamed tables: layer window overflow");
        uint8_t* d = win_[li % 3] + woff_[li];
        woff_[li] += span;
        uint8_t* h = nullptr;
        HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&h), std::max<size_t>(16, nb * B_)));
        host_allocs_.push_back(h);
        stabs_[li].push_back(StreamTab{d, h, nb});
        loaders_.push_back([h, nb, li, name](int b, const GarbledModel& m) {
            const Array& a = m.layers[li].arr(name);
            DASH_CHECK(a.nbytes == nb, "table size mismatch across batch");
            if (a.device_resident() && !a.dev->host)
                HIPCHECK(hipMemcpy(h + nb * b, a.device_ptr(), nb, hipMemcpyDeviceToHost));
            else
                std::memcpy(h + nb * b, a.ptr<uint8_t>(), nb);
        });
        table_bytes_ += nb * B_;
        return reinterpret_cast<const u128*>(d);
    }
    // Op at the start of layer li's ops: layer li - 2 is done (its window may be refilled), layer li + 1's
    // tables go up on the copy stream (layer 0's too, at li = 0), and the evaluation waits for layer li's.
    void stage_layer(size_t li, hipStream_t st) {
        if (li >= 2) HIPCHECK(hipEventRecord(done_[li - 2], st));
        auto issue = [&](size_t x) {
            if (x >= stabs_.size() || stabs_[x].empty()) return;
            if (x >= 3) HIPCHECK(hipStreamWaitEvent(copy_st_, done_[x - 3], 0));
            else if (run_end_recorded_) HIPCHECK(hipStreamWaitEvent(copy_st_, run_end_, 0));  // the previous run's
            for (const auto& t : stabs_[x])
                HIPCHECK(hipMemcpyAsync(t.d, t.h, t.nb * B_, hipMemcpyHostToDevice, copy_st_));
            HIPCHECK(hipEventRecord(ready_[x], copy_st_));
        };
        if (li == 0) issue(0);
        issue(li + 1);
        if (!stabs_[li].empty()) HIPCHECK(hipStreamWaitEvent(st, ready_[li], 0));
    }
    void stage_end(hipStream_t st) {
        HIPCHECK(hipEventRecord(run_end_, st));
        run_end_recorded_ = true;
    }
    void init_streaming(const GarbledModel& m0) {
        const size_t L = m0.layers.size();
        size_t most = 256;
        for (const auto& l : m0.layers) {
            size_t s = 0;
            for (const auto& kv : l.a) s += (kv.second.nbytes * B_ + 255) / 256 * 256;
            most = std::max(most, s);
        }
        win_bytes_ = most;
        for (auto& w : win_) w = dalloc<uint8_t>(win_bytes_);
        woff_.assign(L, 0);
        stabs_.assign(L, {});
        ready_.resize(L);
        done_.resize(L);
        for (auto& e : ready_) HIPCHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        for (auto& e : done_) HIPCHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        HIPCHECK(hipEventCreateWithFlags(&run_end_, hipEventDisableTiming));
        HIPCHECK(hipStreamCreateWithFlags(&copy_st_, hipStreamNonBlocking));
        use_graph_ = false;  // the copy stream's waits on the previous run are issued per run
    }
    // all-zero device rows (the hardened encoding ships no constant labels: public-constant wires have label 0)
    const int16_t* zero_i16(size_t count) {
        int16_t* d = dalloc<int16_t>(count);
        HIPCHECK(hipMemset(d, 0, std::max<size_t>(count * sizeof(int16_t), 64)));
        return d;
    }
    const int16_t* upload_i16_rows(size_t li, const std::string& name) {
        const size_t nb = tmpl_->layers[li].arr(name).nbytes;
        uint8_t* d = dalloc<uint8_t>(nb * B_);
        add_small(d, nb, nb, [nb, li, name](const GarbledModel& m, uint8_t* h) {
            const Array& a = m.layers[li].arr(name);
            DASH_CHECK(a.nbytes == nb, "bias rows size mismatch across batch");
            std::memcpy(h, a.ptr<uint8_t>(), nb);
        });
        return reinterpret_cast<const int16_t*>(d);
    }
    // per-GC concatenated residue labels from model consts ("up.j", "down.s.j", "Z.p")
    const int16_t* upload_const_rows(const std::function<std::string(int)>& name_of) {
        if (hard_) return zero_i16(static_cast<size_t>(B_) * lab_stride_);
        int16_t* d = dalloc<int16_t>(static_cast<size_t>(B_) * lab_stride_);
        std::vector<std::string> names;
        for (int j = 0; j < k_; ++j) names.push_back(name_of(j));
        const int ls = lab_stride_, k = k_;
        std::vector<int> off(lab_off_, lab_off_ + k_), crt = crt_;
        add_small(reinterpret_cast<uint8_t*>(d), sizeof(int16_t) * ls, sizeof(int16_t) * ls,
                  [names, ls, k, off, crt](const GarbledModel& m, uint8_t* hb) {
            int16_t* h = reinterpret_cast<int16_t*>(hb);
            std::fill(h, h + ls, int16_t(0));
            for (int j = 0; j < k; ++j) {
                auto it = m.consts.find(names[j]);
                DASH_CHECK(it != m.consts.end(), "missing model constant " + names[j]);
                std::memcpy(&h[off[j]], it->second.ptr<int16_t>(), sizeof(int16_t) * nr_comps(crt[j]));
            }
        });
        return d;
    }
    CrtInfo crt_info(const std::vector<int>& mods) const {
        CrtInfo c{};
        c.k = static_cast<int>(mods.size());
        int s = 0;
        for (int j = 0; j < c.k; ++j) {
            c.p[j] = mods[j];
            c.n[j] = nr_comps(mods[j]);
            c.prefix[j] = s;
            s += mods[j];
        }
        c.sum = s;
        return c;
    }
    Act act_of(int which) const { return bufs_[which]; }
    void add_op(const std::string& name, std::function<void(hipStream_t)> f) {
        ops_.push_back(std::move(f));
        op_names_.push_back(name);
    }

    // sign gadget phases over `x` (N elements); results in sign scratch
    SignArgs make_sign(size_t li, const std::string& pre, const SignPlan& sp, i64 N, int relu, uint64_t sgate0 = 0,
                       uint64_t mgate0 = 0) {
        SignArgs a{};
        a.hard = hard_ ? 1 : 0;
        a.sgate0 = sgate0;
        a.mgate0 = mgate0;
        a.ny = ny_;
        a.ys = ys_;
        a.crt = crt_info(crt_);
        a.t = static_cast<int>(sp.mrs.size());
        DASH_CHECK(a.t <= kMaxMrs, "MRS base too long for the GPU path");
        for (int d = 0; d < a.t; ++d) a.mrs[d] = sp.mrs[d];
        a.nout = static_cast<int>(sp.out_mod.size());
        for (int o = 0; o < a.nout; ++o) a.out_mod[o] = sp.out_mod[o];
        a.N = N;
        a.B = B_;
        a.n_approx = sp.n_approx;
        a.fused = sp.fused ? 1 : 0;
        a.n_cast = tmpl_->layers[li].arr(pre + "s.cast2").shape[1];
        a.n_sign = sp.n_sign;
        a.approx = upload_tables(li, pre + "s.approx");
        a.cast1 = sp.has_cast1() ? upload_tables(li, pre + "s.cast1") : nullptr;
        a.cast2 = upload_tables(li, pre + "s.cast2");
        a.sign = upload_tables(li, pre + "s.sign");
        a.mrsP = mrsP_;
        a.hx = relu ? hx_ : nullptr;
        a.colx = relu ? colx_ : nullptr;
        a.outP = outP_;
        a.hs = hs_;
        a.cs = cs_;
        a.zc = zc_;
        a.zcol = zcol_;
        a.zc_stride = zstride_;
        a.relu = relu;
        a.csum = csum_;
        {
            int64_t c1 = 0;
            for (int d = a.t - 1; d >= 1; --d) {
                a.c1off[d] = c1;
                c1 += static_cast<int64_t>(k_ + 1) * a.mrs[d];
            }
            // a one-digit MRS base (t = 1) has no casts: the garbler stores a 1-entry placeholder row
            DASH_CHECK(c1 == a.n_cast || (c1 == 0 && a.n_cast <= 1), "cast row size does not match the MRS base");
        }
        int maxn = 0;
        const int k = k_;
        for (size_t d = 1; d < sp.mrs.size(); ++d) maxn = std::max(maxn, nr_comps((k + 1) * sp.mrs[d]));
        maxn = std::max(maxn, nr_comps(sp.mrs[0]));
        DASH_CHECK(maxn <= 64, "MRS moduli too small for the GPU sign chain (label width > 64)");
        sign_maxn_ = maxn;
        return a;
    }

    void build();
    void plan_rescale_legacy(size_t li, i64 iters, i64 N, const CrtInfo& crt, const std::string& lname);

    std::shared_ptr<GarbledModel> tmpl_;  // build() only
    ModelHeader tmpl_h_;
    bool hard_ = false;     // the template's hardened flag (ModelHeader::hardened); every loaded GC must match
    int ny_ = 0;            // y-row pad slots of a ReLU's sign label: k entries + ceil(k / 8) mini pads
    u128* ys_ = nullptr;    // [B][ny][maxSignN] y-row pads (hardened ReLU sign labels)
    size_t tmpl_nlayers_ = 0;
    bool mfma_;
    // streamed tables (stream_table / stage_layer)
    bool stream_ = false;
    struct StreamTab {
        uint8_t* d;  // window address of slot 0 ([B][nb])
        uint8_t* h;  // pinned host copy ([B][nb])
        size_t nb;
    };
    uint8_t* win_[3] = {};
    size_t win_bytes_ = 0;
    std::vector<size_t> woff_;
    std::vector<std::vector<StreamTab>> stabs_;
    hipStream_t copy_st_ = nullptr;
    std::vector<hipEvent_t> ready_, done_;
    hipEvent_t run_end_ = nullptr;
    bool run_end_recorded_ = false;
    std::vector<std::function<void(int, const GarbledModel&)>> loaders_;
    struct SmallLoad {
        size_t off = 0;
        uint8_t* dst0 = nullptr;
        size_t stride = 0, bytes = 0;
        std::function<void(const GarbledModel&, uint8_t*)> fill;
    };
    std::vector<SmallLoad> small_;
    size_t small_bytes_ = 0;
    uint8_t* small_h_ = nullptr;
    uint8_t* small_d_ = nullptr;
    const ScatterDesc* small_desc_ = nullptr;
    hipStream_t load_st_ = nullptr;
    std::mutex load_mu_;  // load(): the staging blocks and load stream above are shared by every slot
    std::map<std::pair<size_t, std::string>, std::pair<uint8_t*, size_t>> arena_;  // (layer, table) -> [B][nb]
    std::vector<int> loaded_;
    int dev_ = 0, B_ = 1, k_ = 0;
    std::vector<int> crt_, out_mod_;
    i64 N0_ = 0, Nout_ = 0;
    std::vector<void*> allocs_, host_allocs_;
    size_t dev_bytes_ = 0, table_bytes_ = 0;
    std::vector<std::function<void(hipStream_t)>> ops_;
    std::vector<std::string> op_names_;
    bool profile_ = false;
    std::vector<hipEvent_t> ev_;
    Act bufs_[4]{};  // ping-pong activation buffers (+ scratch)
    Act final_{};
    Act cur_act_{};
    std::vector<int16_t*> in_stage_;
    std::vector<act_t*> out_stage_;
    std::vector<void*> out_stage_dev_;  // device addresses of the mapped out_stage_ buffers
    bool out_stage_mapped_ = true;
    int16_t* in16_dev_[kMaxRes] = {};  // device int16 copy of the host-encoded inputs (uncompressed input path)
    u128* in_comp_stage_ = nullptr;
    bool use_graph_ = [] {
        const char* e = std::getenv("DASH_HIP_GRAPH");
        return !(e && e[0] == '0');
    }();
    hipGraphExec_t gexec_ = nullptr;
    hipStream_t gstream_ = nullptr;
    long runs_ = 0;
    u128* in_comp_dev_ = nullptr;
    // constants
    ModC* mc_ = nullptr;
    AesGlobals aes_{};
    int lab_stride_ = 0;
    int lab_off_[kMaxRes]{};
    int* d_lab_off_ = nullptr;
    const int16_t* zero_rows_ = nullptr;
    const int16_t* up_rows_ = nullptr;
    u128* mrs_ps_ = nullptr;  // mixed-radix rescale chain scratch (allocated by the first such layer)
    i64 maxSignN_ = 0;
    // planner: a sign-producing rescale whose outputs the next (joint) ReLU's op writes
    bool joint_pending_ = false;
    MrsArgs joint_a_{};
    const u128* zc_ = nullptr;
    const u128* zh_ = nullptr;
    const uint16_t* zcol_ = nullptr;
    int zstride_ = 0;
    // scratch
    u128 *mrsP_ = nullptr, *hx_ = nullptr, *outP_ = nullptr, *hs_ = nullptr, *h0_ = nullptr;
    uint16_t *colx_ = nullptr, *col0_ = nullptr;
    uint8_t* cs_ = nullptr;
    int16_t* csum_ = nullptr;
    int16_t* be_work_ = nullptr;
    int sign_maxn_ = 32;
    std::vector<std::vector<act_t*>> saved_;  // residual-add sources
};

void HipEvaluator::build() {
    const GarbledModel& m0 = *tmpl_;
    hard_ = m0.h.hardened != 0;
    ny_ = k_ + (k_ + 7) / 8;
    // ---- global constants
    const int maxmod = m0.h.max_mod;
    std::vector<ModC> mc(maxmod + 1);
    for (int q = 2; q <= maxmod; ++q) mc[q] = make_modc(q);
    mc_ = upload(mc.data(), mc.size());
    auto te = make_te0();
    auto rk = fixed_round_key_words();
    aes_.te0 = upload(te.data(), te.size());
    aes_.rk = upload(rk.data(), rk.size());
    for (int j = 0; j < k_; ++j) {
        lab_off_[j] = lab_stride_;
        lab_stride_ += nr_comps(crt_[j]);
    }
    d_lab_off_ = upload(lab_off_, k_);
    prepare_zmap(crt_info(crt_));  // VALU dense / conv block lookup, built here (not under a graph capture)
    zero_rows_ = upload_const_rows([&](int j) { return "Z." + std::to_string(crt_[j]); });
    // compressed zero labels + colors for every modulus (carry init)
    zstride_ = maxmod + 1;
    {
        u128* dzc = dalloc<u128>(static_cast<size_t>(B_) * zstride_);
        u128* dzh = dalloc<u128>(static_cast<size_t>(B_) * zstride_);
        uint16_t* dzcol = dalloc<uint16_t>(static_cast<size_t>(B_) * zstride_);
        zc_ = dzc;
        zh_ = dzh;
        zcol_ = dzcol;
        const int zs = zstride_;
        // compressed zero labels, their hashes and colors: one fill writes all three staging blocks (the zc
        // block's fill computes them; the two followers' fills are no-ops on the same pass)
        auto zfill = [zs, maxmod](const GarbledModel& m, u128* zc, u128* zh, uint16_t* zcol) {
            std::fill(zc, zc + zs, u128(0));
            std::fill(zh, zh + zs, u128(0));
            std::fill(zcol, zcol + zs, uint16_t(0));
            LabelBank Z = m.zero_bank();
            for (int q = 2; q <= maxmod; ++q) {
                if (Z.lab[q].empty()) continue;
                zc[q] = compress(Z.lab[q].data(), mod_info(q));
                zh[q] = hash(zc[q]);
                zcol[q] = static_cast<uint16_t>(Z.lab[q][0]);
            }
        };
        const size_t zcb = sizeof(u128) * zs, zcolb = sizeof(uint16_t) * zs;
        const size_t zoff = small_bytes_;  // the three blocks are staged back to back (16-B rounded)
        const size_t zhoff = zoff + (zcb + 15) / 16 * 16, zcoloff = zhoff + (zcb + 15) / 16 * 16;
        add_small(reinterpret_cast<uint8_t*>(dzc), zcb, zcb, [zfill, zoff, zhoff, zcoloff](const GarbledModel& m, uint8_t* h) {
            zfill(m, reinterpret_cast<u128*>(h), reinterpret_cast<u128*>(h + (zhoff - zoff)),
                  reinterpret_cast<uint16_t*>(h + (zcoloff - zoff)));
        });
        add_small(reinterpret_cast<uint8_t*>(dzh), zcb, zcb, [](const GarbledModel&, uint8_t*) {});
        add_small(reinterpret_cast<uint8_t*>(dzcol), zcolb, zcolb, [](const GarbledModel&, uint8_t*) {});
    }
    bool any_rescale = false;
    for (auto& l : m0.layers) any_rescale |= (l.kind == K_RESCALE && l.param("mode", 0) != 2);  // mode 2: no shift labels
    if (any_rescale) up_rows_ = upload_const_rows([&](int j) { return "up." + std::to_string(j); });

    // ---- shape pass: buffer capacities
    N0_ = 1;
    for (auto d : m0.h.in_dims) N0_ *= d;
    i64 maxN = N0_, maxSignN = 1, maxPoolSlots = 1;
    std::vector<int> widest(k_, 0), mods = crt_;
    for (int j = 0; j < k_; ++j) widest[j] = nr_comps(crt_[j]);
    {
        i64 N = N0_;
        std::vector<i64> outN(m0.layers.size() + 1, N0_);
        size_t li0 = 0;
        for (auto& l : m0.layers) {
            if (l.p.count("in_src")) N = outN[l.param("in_src") + 1];
            switch (l.kind) {
                case K_DENSE: N = l.param("out"); break;
                case K_CONV: N = ConvGeom(l).out_size(); break;
                case K_RELU: case K_SIGN: case K_RESCALE: maxSignN = std::max(maxSignN, N); break;
                case K_MAXPOOL: {
                    PoolGeom G(l.p);
                    maxPoolSlots = std::max(maxPoolSlots, G.out_size() * G.kh * G.kw);
                    maxSignN = std::max(maxSignN, G.out_size() * G.kh * G.kw);
                    N = G.out_size();
                    break;
                }
                case K_MAX:
                    maxPoolSlots = std::max(maxPoolSlots, N);
                    maxSignN = std::max(maxSignN, N);
                    N = 1;
                    break;
                case K_SUMPOOL: N = PoolGeom(l.p).out_size(); break;
                case K_MULT: case K_MMULT: N /= 2; break;
                case K_PROJ: {
                    const auto& om = l.vec("out_mod");
                    for (int j = 0; j < k_; ++j) widest[j] = std::max(widest[j], nr_comps(static_cast<int>(om[j])));
                    break;
                }
                default: break;
            }
            maxN = std::max(maxN, N);
            outN[++li0] = N;
        }
    }
    const i64 cap = std::max(maxN, maxPoolSlots);
    for (int bi = 0; bi < 4; ++bi) {
        bufs_[bi].N = 0;
        for (int j = 0; j < k_; ++j) {
            // + 64 B: the MFMA dense kernel reads whole 16-byte k slices past the last column's end
            const size_t count = static_cast<size_t>(B_) * widest[j] * cap + 64;
            bufs_[bi].p[j] = dalloc<act_t>(count);
            // defined contents before any input is staged (serving primes the hipGraph with an unencoded run)
            HIPCHECK(hipMemset(bufs_[bi].p[j], 0, count * sizeof(act_t)));
        }
    }
    int tmax = std::max<int>(1, static_cast<int>(m0.h.mrs.size()));
    mrsP_ = dalloc<u128>(static_cast<size_t>(B_) * k_ * tmax * maxSignN);
    hx_ = dalloc<u128>(static_cast<size_t>(B_) * k_ * maxSignN);
    csum_ = dalloc<int16_t>(static_cast<size_t>(B_) * tmax * kCsumComps * maxSignN);
    colx_ = dalloc<uint16_t>(static_cast<size_t>(B_) * k_ * maxSignN);
    outP_ = dalloc<u128>(static_cast<size_t>(B_) * k_ * maxSignN);
    maxSignN_ = maxSignN;
    hs_ = dalloc<u128>(static_cast<size_t>(B_) * maxSignN);
    if (hard_) ys_ = dalloc<u128>(static_cast<size_t>(B_) * ny_ * maxSignN);
    cs_ = dalloc<uint8_t>(static_cast<size_t>(B_) * maxSignN);
    h0_ = dalloc<u128>(static_cast<size_t>(B_) * maxN);
    col0_ = dalloc<uint16_t>(static_cast<size_t>(B_) * maxN);
    for (int j = 0; j < k_; ++j) {
        int16_t* p = nullptr;
        HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&p), sizeof(int16_t) * B_ * nr_comps(crt_[j]) * N0_));
        host_allocs_.push_back(p);
        in_stage_.push_back(p);
    }

    // ---- plan
    std::vector<int> keep(m0.layers.size() + 1, 0);
    for (auto& l : m0.layers) {
        if (l.kind == K_ADD) keep[l.param("src") + 1] = 1;
        if (l.p.count("in_src")) keep[l.param("in_src") + 1] = 1;
    }
    saved_.assign(m0.layers.size() + 1, {});
    std::vector<i64> saved_n(m0.layers.size() + 1, 0);
    std::vector<std::vector<int>> saved_mods(m0.layers.size() + 1);
    int cur = 0;  // buffer index holding the current activation
    i64 N = N0_;
    const CrtInfo crt = crt_info(crt_);
    auto save_if_needed = [&](size_t slot, int buf, i64 n_el, const std::vector<int>& md) {
        if (!keep[slot]) return;
        std::vector<act_t*> s;
        for (int j = 0; j < k_; ++j) {
            const size_t bytes = sizeof(act_t) * B_ * nr_comps(md[j]) * n_el;
            act_t* d = dalloc<act_t>(bytes / sizeof(act_t));
            act_t* src = bufs_[buf].p[j];
            add_op("save", [d, src, bytes](hipStream_t st) { HIPCHECK(hipMemcpyAsync(d, src, bytes, hipMemcpyDeviceToDevice, st)); });
            s.push_back(d);
        }
        saved_[slot] = s;
        saved_n[slot] = n_el;
        saved_mods[slot] = md;
    };
    save_if_needed(0, cur, N, mods);
    if (stream_) init_streaming(m0);

    for (size_t li = 0; li < m0.layers.size(); ++li) {
        const GLayer& g = m0.layers[li];
        if (stream_) add_op("stage", [this, li](hipStream_t st) { stage_layer(li, st); });
        const int nxt = (cur + 1) % 2;
        const std::string lname = std::string(kind_name(g.kind)) + "#" + std::to_string(li);
        if (g.p.count("in_src")) {
            // layer reads an earlier output (projection shortcut): restore it into the current buffer
            const i64 src = g.param("in_src");
            const auto& sv = saved_[src + 1];
            DASH_CHECK(!sv.empty(), "in_src source not saved");
            N = saved_n[src + 1];
            mods = saved_mods[src + 1];
            for (int j = 0; j < k_; ++j) {
                const size_t bytes = sizeof(act_t) * B_ * nr_comps(mods[j]) * N;
                act_t* d = bufs_[cur].p[j];
                const act_t* sp = sv[j];
                add_op("restore", [d, sp, bytes](hipStream_t st) {
                    HIPCHECK(hipMemcpyAsync(d, sp, bytes, hipMemcpyDeviceToDevice, st));
                });
            }
        }
        cur_act_ = act_of(cur);
        switch (g.kind) {
            case K_FLATTEN:
                break;
            case K_DENSE: {
                DenseArgs a{};
                a.crt = crt;
                a.K = g.param("in");
                a.O = g.param("out");
                const i64 ch = g.param("channel_tf", 0);
                const Array& w = g.arr("w");
                for (int j = 0; j < k_; ++j) {
                    const int p = crt_[j];
                    std::vector<int16_t> wt(static_cast<size_t>(a.K * a.O));
                    std::vector<int32_t> zc(a.O, 0);
                    for (i64 o = 0; o < a.O; ++o)
                        for (i64 i = 0; i < a.K; ++i) {
                            const int v = static_cast<int>(w.ptr<i64>()[o * a.K + i] % p);
                            wt[i * a.O + o] = static_cast<int16_t>(v);
                            if (v == 0) ++zc[o];
                        }
                    a.w[j] = upload(wt.data(), wt.size());
                    a.zc[j] = upload(zc.data(), zc.size());
                    a.bias[j] = hard_ ? zero_i16(static_cast<size_t>(B_) * a.O * nr_comps(p))
                                      : upload_i16_rows(li, arr_name("bias.", j, ""));
                }
                // MFMA path: centered int8 weights [O][Kpad], channel_tf folded into the column order
                a.Kpad = static_cast<int>((a.K + 63) / 64 * 64);
                bool mfma_ok = mfma_ && a.K < (1 << 17);  // 127 * 127 * K fits the int32 accumulator
                for (int j = 0; j < k_; ++j) mfma_ok = mfma_ok && crt_[j] <= 255;
                for (int j = 0; j < k_; ++j) {
                    a.w8[j] = nullptr;
                    if (!mfma_ok) continue;
                    const int p = crt_[j];
                    std::vector<int8_t> w8(static_cast<size_t>(a.O) * a.Kpad, 0);
                    for (i64 o = 0; o < a.O; ++o)
                        for (i64 i = 0; i < a.K; ++i) {
                            const int v = static_cast<int>(w.ptr<i64>()[o * a.K + i] % p);
                            const i64 s = ch > 0 ? dense_src(i, a.K, ch) : i;
                            w8[static_cast<size_t>(o) * a.Kpad + s] = static_cast<int8_t>(v > p / 2 ? v - p : v);
                        }
                    a.w8[j] = upload(w8.data(), w8.size());
                }
                a.zero = zero_rows_;
                a.lab_stride = lab_stride_;
                for (int j = 0; j < k_; ++j) a.lab_off[j] = lab_off_[j];
                if (ch > 0) {
                    std::vector<int32_t> src(a.K);
                    for (i64 i = 0; i < a.K; ++i) src[i] = static_cast<int32_t>(dense_src(i, a.K, ch));
                    a.src = upload(src.data(), src.size());
                }
                Act x = act_of(cur), y = act_of(nxt);
                x.N = N;
                y.N = a.O;
                const int B = B_;
                add_op(lname, [a, x, y, B](hipStream_t st) { launch_dense(a, x, y, B, st); });
                N = a.O;
                cur = nxt;
                break;
            }
            case K_CONV: {
                ConvGeom G(g);
                ConvArgs a{};
                a.crt = crt;
                a.C = static_cast<int>(G.C); a.H = static_cast<int>(G.H); a.W = static_cast<int>(G.W);
                a.F = static_cast<int>(G.F); a.kh = static_cast<int>(G.kh); a.kw = static_cast<int>(G.kw);
                a.sh = static_cast<int>(G.sh); a.sw = static_cast<int>(G.sw);
                a.ph = static_cast<int>(G.ph); a.pw = static_cast<int>(G.pw);
                a.OH = static_cast<int>(G.OH); a.OW = static_cast<int>(G.OW);
                const i64 K = G.K();
                a.Kpad = static_cast<int>((K + 63) / 64 * 64);
                a.use_mfma = mfma_ ? 1 : 0;
                // LDS-image kernel geometry: 64-channel chunks, row bands that fit 64 KiB of LDS
                {
                    static const bool img_ok = [] {
                        const char* e = std::getenv("DASH_CONV_IMG");
                        return !(e && e[0] == '0');
                    }();
                    int max_p = 0;
                    for (int j = 0; j < k_; ++j) max_p = std::max(max_p, crt_[j]);
                    conv_plan(a, max_p, mfma_ && img_ok);
                    if (!(mfma_ && img_ok)) a.band = a.nbands = 0;
                }
                a.img_off[0] = 0;
                for (int j = 0; j < k_; ++j) a.img_off[j + 1] = a.img_off[j] + static_cast<i64>(B_) * crt.n[j];
                const Array& w = g.arr("w");
                for (int j = 0; j < k_; ++j) {
                    const int p = crt_[j];
                    std::vector<int16_t> wm(static_cast<size_t>(G.F * K));
                    std::vector<int8_t> w8(static_cast<size_t>(G.F) * a.Kpad, 0);
                    std::vector<int32_t> zc(G.F, 0);
                    for (i64 f = 0; f < G.F; ++f)
                        for (i64 q = 0; q < K; ++q) {
                            const int v = static_cast<int>(w.ptr<i64>()[f * K + q] % p);
                            wm[f * K + q] = static_cast<int16_t>(v);
                            if (v == 0) ++zc[f];
                            w8[f * a.Kpad + q] = static_cast<int8_t>(v > p / 2 ? v - p : v);
                        }
                    a.w[j] = upload(wm.data(), wm.size());
                    a.w8[j] = (mfma_ && p <= 255) ? upload(w8.data(), w8.size()) : nullptr;
                    if (a.nbands > 0 && p <= 255) {
                        // [F16][kh][kw][Cpad] centered int8 (im2col order ci*kh*kw + dy*kw + dx -> (dy, dx, ci))
                        const std::vector<int8_t> w8r = conv_w8r(a, w8, static_cast<int>(G.F));
                        a.w8r[j] = upload(w8r.data(), w8r.size());
                    } else {
                        a.w8r[j] = nullptr;
                    }
                    a.zc[j] = upload(zc.data(), zc.size());
                    a.bias[j] = hard_ ? zero_i16(static_cast<size_t>(B_) * G.F * nr_comps(p))
                                      : upload_i16_rows(li, arr_name("bias.", j, ""));
                }
                a.zero = zero_rows_;
                a.lab_stride = lab_stride_;
                for (int j = 0; j < k_; ++j) a.lab_off[j] = lab_off_[j];
                Act x = act_of(cur), y = act_of(nxt);
                const int B = B_;
                add_op(lname, [a, x, y, B](hipStream_t st) { launch_conv(a, x, y, B, st); });
                N = G.out_size();
                cur = nxt;
                break;
            }
            case K_RELU: {
                if (g.param("smode", 0) == 2) {  // sign from the preceding rescale (RescaleMrsPlan::sign_last)
                    DASH_CHECK(li > 0 && m0.layers[li - 1].kind == K_RESCALE &&
                                   m0.layers[li - 1].param("sign_out", 0) == 1,
                               "joint ReLU must follow a sign-producing rescale");
                    SignArgs sa{};
                    sa.crt = crt;
                    sa.N = N;
                    sa.B = B_;
                    sa.hx = hx_;
                    sa.colx = colx_;
                    sa.hs = hs_;
                    sa.cs = cs_;
                    sa.hard = hard_ ? 1 : 0;
                    sa.mgate0 = gate_base(li + 1, 2);
                    sa.ny = ny_;
                    sa.ys = ys_;
                    const u128* gt = upload_tables(li, "mm.g");
                    const u128* et = upload_tables(li, "mm.e");
                    Act x = act_of(cur), y = act_of(nxt);
                    const ModC* mc = mc_;
                    const AesGlobals ag = aes_;
                    const int B = B_;
                    if (joint_pending_) {
                        const MrsArgs ma = joint_a_;
                        joint_pending_ = false;
                        add_op(lname + ".C", [ma, sa, x, y, gt, et, B, mc, ag](hipStream_t st) {
                            launch_rescale_relu_out(ma, sa, x, y, gt, et, B, mc, ag, st);
                        });
                    } else {
                        add_op(lname + ".C", [sa, x, y, gt, et, B, mc, ag](hipStream_t st) {
                            launch_relu_joint(sa, x, y, gt, et, B, mc, ag, st);
                        });
                    }
                    cur = nxt;
                    break;
                }
                if (g.param("smode", 0) == 1) {  // exact mixed-radix sign (gadgets.h SignMrsPlan)
                    const SignMrsPlan P(crt_);
                    MrsArgs a{};
                    a.crt = crt;
                    a.N = N;
                    a.n_tab = g.arr("mrs").shape[1];
                    a.tab = upload_tables(li, "mrs");
                    for (int i = 0; i + 1 < k_; ++i) a.dig_off[i] = P.dig_off[i];
                    if (!mrs_ps_) mrs_ps_ = dalloc<u128>(static_cast<size_t>(B_) * std::max(1, k_ * (k_ - 1) / 2) * maxSignN_);
                    a.ps = mrs_ps_;
                    a.mode = 1;
                    a.hs = hs_;
                    a.cs = cs_;
                    DASH_CHECK(hard_, "the mixed-radix sign exists in the hardened encoding only");
                    a.gate0 = gate_base(li + 1, 1);
                    a.rgate0 = gate_base(li + 1, 2);
                    a.ny = ny_;
                    a.ys = ys_;
                    SignArgs sa{};
                    sa.crt = crt;
                    sa.N = N;
                    sa.B = B_;
                    sa.hx = hx_;
                    sa.colx = colx_;
                    sa.hs = hs_;
                    sa.cs = cs_;
                    sa.hard = 1;
                    sa.mgate0 = gate_base(li + 1, 2);
                    sa.ny = ny_;
                    sa.ys = ys_;
                    const u128* gt = upload_tables(li, "mm.g");
                    const u128* et = upload_tables(li, "mm.e");
                    Act x = act_of(cur), y = act_of(nxt);
                    const ModC* mc = mc_;
                    const AesGlobals ag = aes_;
                    const int B = B_;
                    add_op(lname + ".mrs", [a, sa, x, y, gt, et, B, mc, ag](hipStream_t st) {
                        launch_relu_mrs(a, sa, x, y, gt, et, B, mc, ag, st);
                    });
                    cur = nxt;
                    break;
                }
                SignPlan sp(crt_, m0.h.mrs, {2}, 0, 1, m0.h.sign_fused != 0);
                SignArgs a = make_sign(li, "", sp, N, 1, gate_base(li + 1, 1), gate_base(li + 1, 2));
                const u128* gt = upload_tables(li, "mm.g");
                const u128* et = upload_tables(li, "mm.e");
                Act x = act_of(cur), y = act_of(nxt);
                const ModC* mc = mc_;
                const AesGlobals ag = aes_;
                const int maxn = sign_maxn_;
                add_op(lname + ".A", [a, x, mc, ag](hipStream_t st) { launch_sign_approx(a, x, mc, ag, st); });
                add_op(lname + ".B", [a, maxn, mc, ag](hipStream_t st) { launch_sign_chain(a, maxn, mc, ag, st); });
                add_op(lname + ".C", [a, x, y, gt, et, mc](hipStream_t st) { launch_relu_mult(a, x, y, gt, et, mc, st); });
                cur = nxt;
                break;
            }
            case K_SIGN: {
                SignPlan sp(crt_, m0.h.mrs, crt_, -1, 1, m0.h.sign_fused != 0);
                SignArgs a = make_sign(li, "", sp, N, 0, gate_base(li + 1, 1), 0);
                Act x = act_of(cur), y = act_of(nxt);
                const ModC* mc = mc_;
                const AesGlobals ag = aes_;
                const int maxn = sign_maxn_;
                const int B = B_;
                const u128* outP = outP_;
                const i64 NN = N;
                add_op(lname + ".A", [a, x, mc, ag](hipStream_t st) { launch_sign_approx(a, x, mc, ag, st); });
                add_op(lname + ".B", [a, maxn, mc, ag](hipStream_t st) { launch_sign_chain(a, maxn, mc, ag, st); });
                add_op(lname + ".unpack", [outP, y, crt, mc, NN, B](hipStream_t st) { launch_unpack(outP, crt.k, y, crt, mc, NN, B, st); });
                cur = nxt;
                break;
            }
            case K_RESCALE: {
                const i64 mode = g.param("mode", 0);
                const i64 iters = g.param("iters");
                if (mode == 2) {  // mixed-radix construction of the legacy function (gadgets.h RescaleMrsPlan)
                    const bool so = g.param("sign_out", 0) == 1;  // joint: the next ReLU's sign -> hs_, cs_
                    const RescaleMrsPlan P(crt_, static_cast<int>(g.param("l")), so);
                    DASH_CHECK(P.T <= m0.h.max_mod, "model lacks the mod-2^(l+1) label constants");
                    MrsArgs a{};
                    a.crt = crt;
                    a.T = static_cast<int>(P.T);
                    a.N = N;
                    a.n_tab = P.n_tab;
                    a.tab = upload_tables(li, "mrs");
                    for (int i = 0; i < k_; ++i) {
                        a.dig_off[i] = P.dig_off[i];
                        a.sinv[i] = static_cast<int>(P.Sinv[i]);
                    }
                    a.fin_off = P.fin_off;
                    const int bits = P.l + 1, nf = nr_comps(static_cast<int>(P.T));
                    a.hmask = 0;
                    for (int f = 0; f < nf; ++f) a.hmask |= static_cast<u128>(1) << (bits * f + bits - 1);
                    a.pf = outP_;  // [B][k][N] <= the sign outputs' scratch
                    if (!mrs_ps_) mrs_ps_ = dalloc<u128>(static_cast<size_t>(B_) * std::max(1, k_ * (k_ - 1) / 2) * maxSignN_);
                    a.ps = mrs_ps_;
                    a.mode = so ? 2 : 0;
                    a.hs = hs_;
                    a.cs = cs_;
                    a.hx = hx_;
                    a.colx = colx_;
                    DASH_CHECK(hard_, "the mixed-radix rescale exists in the hardened encoding only");
                    a.gate0 = gate_base(li + 1, 30);
                    a.rgate0 = so ? gate_base(li + 2, 2) : 0;  // the joint ReLU (next layer)'s half gates
                    a.ny = ny_;
                    a.ys = ys_;
                    Act x = act_of(cur);
                    const ModC* mc = mc_;
                    const AesGlobals ag = aes_;
                    const int B = B_;
                    // joint ReLU next and this output not kept for a later layer: the ReLU's op can write both
                    // outputs in one pass (k_rescale_relu_out), here only the chain runs. Measured (MiniONN):
                    // faster at batch 1 (2.81 vs 2.98 ms per step), slower at batch 24 (15.9 vs 15.1 ms: the
                    // hash -> second pass dependency per lane), so only small batches take it;
                    // DASH_JOINT_FUSE=0/1 forces it off/on.
                    static const int fuse_env = [] {
                        const char* e = std::getenv("DASH_JOINT_FUSE");
                        return e ? std::atoi(e) : -1;
                    }();
                    // Round 4 (AES tables) had the two staged kernels ahead at batch 1 for N % 16 == 0; with the
                    // hardened encoding the fused form wins there too (latency_b1 2.21 -> 2.14 ms) and ties at
                    // 24 GCs (9.85 vs 9.82 ms per step, profiles/ab/r5_joint_fuse_*.json): on for batch <= 2.
                    const bool fuse = fuse_env >= 0 ? fuse_env == 1 : B_ <= 2;
                    const bool defer = fuse && so && li + 1 < m0.layers.size() && m0.layers[li + 1].kind == K_RELU &&
                                       m0.layers[li + 1].param("smode", 0) == 2 && !keep[li + 1] &&
                                       !m0.layers[li + 1].p.count("in_src");
                    if (defer) {
                        joint_a_ = a;
                        joint_pending_ = true;
                    }
                    add_op(lname + ".mrs", [a, x, B, mc, ag, defer](hipStream_t st) {
                        launch_rescale_mrs(a, x, B, mc, ag, st, defer);
                    });
                    break;
                }
                if (mode == 0) {
                    plan_rescale_legacy(li, iters, N, crt, lname);
                    break;
                }
                for (i64 it = 0; it < iters; ++it) {
                    std::vector<int> factors;
                    if (mode == 0)
                        factors = {2};
                    else
                        for (auto v : g.vec("s")) factors.push_back(static_cast<int>(v));
                    RescalePlan P(crt_, m0.h.mrs, factors, mode == 0, m0.h.sign_fused != 0);
                    const std::string pre = arr_name("it", static_cast<int>(it), ".");
                    const u128* trans = upload_tables(li, pre + "trans");
                    Act x = act_of(cur);
                    const ModC* mc = mc_;
                    const AesGlobals ag = aes_;
                    const int B = B_;
                    const i64 NN = N;
                    i64 off = 0;
                    for (size_t f = 0; f < P.factors.size(); ++f) {
                        const int fi = P.factor_idx[f], s = P.factors[f];
                        const int add_up = f == 0 ? 1 : 0;
                        const int16_t* up = up_rows_ + lab_off_[fi];
                        u128* h0 = h0_;
                        uint16_t* col0 = col0_;
                        const int ls = lab_stride_;
                        const int hd = hard_ ? 1 : 0;
                        add_op(lname + ".hash", [x, fi, s, up, ls, add_up, NN, B, h0, col0, mc, ag, hd](hipStream_t st) {
                            launch_rescale_hash(x, fi, s, up, ls, add_up, NN, B, h0, col0, mc, ag, st, hd);
                        });
                        RescaleArgs ra{};
                        ra.crt = crt;
                        ra.N = N;
                        ra.fi = fi;
                        ra.s = s;
                        ra.add_up = add_up;
                        for (size_t q = 0; q < P.active[f].size(); ++q) {
                            const int jj = P.active[f][q];
                            ra.active[jj] = 1;
                            ra.aidx[jj] = static_cast<int>(q);
                            ra.inv[jj] = static_cast<int>(P.inv[f][q]);
                        }
                        ra.n_trans = P.n_trans;
                        ra.off = off;
                        off += static_cast<i64>(P.active[f].size()) * s;
                        ra.trans = trans;
                        ra.h0 = h0_;
                        ra.col0 = col0_;
                        ra.up = up_rows_;
                        ra.zero = zero_rows_;
                        ra.lab_stride = lab_stride_;
                        for (int j = 0; j < k_; ++j) ra.lab_off[j] = lab_off_[j];
                        ra.hard = hard_ ? 1 : 0;
                        ra.gate0 = gate_base(li + 1, 10 + it);
                        ra.factor = static_cast<int>(f);
                        add_op(lname + ".update", [ra, x, B, mc](hipStream_t st) { launch_rescale_update(ra, x, B, mc, st); });
                    }
                    const u128* signP = nullptr;
                    if (P.sign_be) {
                        SignArgs a = make_sign(li, pre, P.sign, N, 0);
                        const int maxn = sign_maxn_;
                        add_op(lname + ".sA", [a, x, mc, ag](hipStream_t st) { launch_sign_approx(a, x, mc, ag, st); });
                        add_op(lname + ".sB", [a, maxn, mc, ag](hipStream_t st) { launch_sign_chain(a, maxn, mc, ag, st); });
                        signP = outP_;
                    } else {
                        const BEPlan& be = P.be;
                        BEArgs ba{};
                        ba.E = static_cast<int>(be.moduli.size());
                        ba.nonext = be.nonext;
                        std::vector<int> idx(ba.E);
                        for (int i = 0; i < ba.E; ++i) idx[be.pos_of[i]] = i;
                        for (int i = 0; i < ba.E; ++i) {
                            ba.swapped[i] = be.swapped[i];
                            ba.src[i] = idx[i];
                        }
                        for (int i = 0; i + 1 < ba.E; ++i)
                            for (size_t jj = 0; jj < be.inv_partial[i].size(); ++jj)
                                ba.inv[i][jj] = static_cast<int>(be.inv_partial[i][jj]);
                        ba.nextra = static_cast<int>(be.extra.size());
                        for (int xi = 0; xi < ba.nextra; ++xi) {
                            ba.extra_res[xi] = be.extra_idx[xi];
                            ba.extra_pos[xi] = be.pos_of[be.extra_idx[xi]];
                            const int q = be.moduli[be.extra_idx[xi]];
                            ba.invv[xi] = static_cast<int>(pmod(-be.invv[xi], q));
                        }
                        ba.N = N;
                        ba.n_tab = be.n_tab;
                        ba.tab = upload_tables(li, pre + "be");
                        if (!be_work_) be_work_ = dalloc<int16_t>(static_cast<size_t>(B_) * k_ * 128 * maxN);
                        ba.work = be_work_;
                        ba.hard = hard_ ? 1 : 0;
                        ba.gate0 = gate_base(li + 1, 10 + it);
                        add_op(lname + ".be", [ba, x, B, mc, ag](hipStream_t st) { launch_base_ext(ba, x, B, mc, ag, st); });
                    }
                    const int16_t* down = upload_const_rows(
                        [&](int j) { return "down." + std::to_string(P.sprod) + "." + std::to_string(j); });
                    const int ls = lab_stride_;
                    const int* loff = d_lab_off_;
                    add_op(lname + ".post", [x, crt, NN, B, signP, down, ls, loff, mc](hipStream_t st) {
                        launch_rescale_post(x, crt, NN, B, signP, down, ls, loff, mc, st);
                    });
                }
                break;
            }
            case K_MAXPOOL:
            case K_MAX: {
                i64 Nout, K;
                std::vector<i64> idx;
                if (g.kind == K_MAXPOOL) {
                    PoolGeom G(g.p);
                    Nout = G.out_size();
                    K = G.kh * G.kw;
                    std::vector<i64> w;
                    for (i64 o = 0; o < Nout; ++o) {
                        G.window(o, w);
                        idx.insert(idx.end(), w.begin(), w.end());
                    }
                } else {
                    Nout = 1;
                    K = N;
                    for (i64 i = 0; i < N; ++i) idx.push_back(i);
                }
                const int64_t* didx = upload(idx.data(), idx.size());
                MaxTree T(K);
                SignPlan sp(crt_, m0.h.mrs, {2}, 0, 1, m0.h.sign_fused != 0);
                // buffers: vals in 2/3 ping-pong, diff in nxt-other... use bufs 2,3 for vals; relu out in buf nxt
                int va = 2, vb = 3;
                Act xin = act_of(cur), v0 = act_of(va);
                const int B = B_;
                const i64 NN = N;
                add_op(lname + ".gather", [xin, NN, v0, Nout, K, didx, crt, B](hipStream_t st) {
                    launch_copy_gather(xin, NN, v0, Nout * K, didx, crt, B, st);
                });
                // scratch for diffs: reuse buffer `cur` (its content is no longer needed) and relu out in `nxt`
                for (size_t lv = 0; lv < T.ops.size(); ++lv) {
                    const int ops = T.ops[lv], cnt = T.cnt[lv], cnt1 = T.cnt[lv + 1];
                    const std::string pre = arr_name("lv", static_cast<int>(lv), ".");
                    SignArgs a = make_sign(li, pre, sp, Nout * ops, 1, gate_base(li + 1, 20 + 2 * lv),
                                           gate_base(li + 1, 21 + 2 * lv));
                    const u128* gt = upload_tables(li, pre + "mm.g");
                    const u128* et = upload_tables(li, pre + "mm.e");
                    Act V = act_of(va), D = act_of(cur), Rr = act_of(nxt), NV = act_of(vb);
                    const ModC* mc = mc_;
                    const AesGlobals ag = aes_;
                    const int maxn = sign_maxn_;
                    const i64 Nv = Nout * cnt;
                    add_op(lname + ".diff", [V, Nv, D, Nout, ops, cnt, crt, B](hipStream_t st) {
                        launch_pair_diff(V, Nv, D, Nout, ops, cnt, crt, B, st);
                    });
                    add_op(lname + ".A", [a, D, mc, ag](hipStream_t st) { launch_sign_approx(a, D, mc, ag, st); });
                    add_op(lname + ".B", [a, maxn, mc, ag](hipStream_t st) { launch_sign_chain(a, maxn, mc, ag, st); });
                    add_op(lname + ".C", [a, D, Rr, gt, et, mc](hipStream_t st) { launch_relu_mult(a, D, Rr, gt, et, mc, st); });
                    add_op(lname + ".add", [V, Nv, Rr, NV, Nout, ops, cnt, cnt1, crt, B](hipStream_t st) {
                        launch_pair_add(V, Nv, Rr, NV, Nout, ops, cnt, cnt1, crt, B, st);
                    });
                    std::swap(va, vb);
                }
                // result (cnt == 1) lives in buffer va: copy into nxt
                std::vector<i64> ident(Nout);
                for (i64 o = 0; o < Nout; ++o) ident[o] = o;
                const int64_t* did = upload(ident.data(), ident.size());
                Act vres = act_of(va), y = act_of(nxt);
                add_op(lname + ".out", [vres, Nout, y, did, crt, B](hipStream_t st) {
                    launch_copy_gather(vres, Nout, y, Nout, did, crt, B, st);
                });
                N = Nout;
                cur = nxt;
                break;
            }
            case K_SUMPOOL: {
                PoolGeom G(g.p);
                std::vector<i64> idx, w;
                for (i64 o = 0; o < G.out_size(); ++o) {
                    G.window(o, w);
                    idx.insert(idx.end(), w.begin(), w.end());
                }
                const int64_t* didx = upload(idx.data(), idx.size());
                Act x = act_of(cur), y = act_of(nxt);
                const i64 NN = N, No = G.out_size();
                const int K = static_cast<int>(G.kh * G.kw);
                const int B = B_;
                add_op(lname, [x, NN, y, No, didx, K, crt, B](hipStream_t st) { launch_window_sum(x, NN, y, No, didx, K, crt, B, st); });
                N = No;
                cur = nxt;
                break;
            }
            case K_ADD: {
                const i64 src = g.param("src");
                const auto& s = saved_[src + 1];
                DASH_CHECK(!s.empty(), "residual source not saved");
                Act x = act_of(cur), y{};
                for (int j = 0; j < k_; ++j) y.p[j] = s[j];
                const i64 NN = N;
                const int B = B_;
                add_op(lname, [x, y, NN, crt, B](hipStream_t st) { launch_add(x, y, NN, crt, B, st); });
                break;
            }
            case K_PROJ: {
                const auto& inm = g.vec("in_mod");
                const auto& outm = g.vec("out_mod");
                ProjArgs a{};
                a.k = k_;
                a.N = N;
                a.hard = hard_ ? 1 : 0;
                a.gate0 = gate_base(li + 1, 1);
                for (int j = 0; j < k_; ++j) {
                    a.pin[j] = static_cast<int>(inm[j]);
                    a.pout[j] = static_cast<int>(outm[j]);
                    a.tab[j] = upload_tables(li, arr_name("t.", j, ""));
                    mods[j] = a.pout[j];
                }
                Act x = act_of(cur), y = act_of(nxt);
                const ModC* mc = mc_;
                const AesGlobals ag = aes_;
                const int B = B_;
                add_op(lname, [a, x, y, B, mc, ag](hipStream_t st) { launch_proj(a, x, y, B, mc, ag, st); });
                cur = nxt;
                break;
            }
            case K_MULT:
            case K_MMULT: {
                MultArgs a{};
                a.crt = crt;
                a.No = N / 2;
                a.hard = hard_ ? 1 : 0;
                a.gate0 = gate_base(li + 1, 1);
                a.q = g.kind == K_MMULT ? static_cast<int>(g.param("q")) : 0;
                if (a.q) a.t = upload_tables(li, "t");
                a.g = upload_tables(li, "g");
                a.e = upload_tables(li, "e");
                Act x = act_of(cur), y = act_of(nxt);
                const ModC* mc = mc_;
                const AesGlobals ag = aes_;
                const int B = B_;
                add_op(lname, [a, x, y, B, mc, ag](hipStream_t st) { launch_mult(a, x, y, B, mc, ag, st); });
                N = a.No;
                cur = nxt;
                break;
            }
            case K_BASEEXT: {
                std::vector<int> ext;
                for (auto v : g.vec("extra")) ext.push_back(static_cast<int>(v));
                BEPlan be(crt_, ext);
                Act x = act_of(cur);
                const ModC* mc = mc_;
                const AesGlobals ag = aes_;
                const int B = B_;
                for (int xi : be.extra_idx) {
                    RescaleArgs ra{};
                    ra.crt = crt;
                    ra.N = N;
                    ra.fi = xi;
                    ra.zero = zero_rows_;
                    ra.up = zero_rows_;
                    ra.lab_stride = lab_stride_;
                    for (int j = 0; j < k_; ++j) ra.lab_off[j] = lab_off_[j];
                    add_op(lname + ".zero", [ra, x, B, mc](hipStream_t st) { launch_rescale_update(ra, x, B, mc, st); });
                }
                BEArgs ba{};
                ba.E = static_cast<int>(be.moduli.size());
                ba.nonext = be.nonext;
                std::vector<int> idx(ba.E);
                for (int i = 0; i < ba.E; ++i) idx[be.pos_of[i]] = i;
                for (int i = 0; i < ba.E; ++i) {
                    ba.swapped[i] = be.swapped[i];
                    ba.src[i] = idx[i];
                }
                for (int i = 0; i + 1 < ba.E; ++i)
                    for (size_t jj = 0; jj < be.inv_partial[i].size(); ++jj) ba.inv[i][jj] = static_cast<int>(be.inv_partial[i][jj]);
                ba.nextra = static_cast<int>(be.extra.size());
                for (int xi = 0; xi < ba.nextra; ++xi) {
                    ba.extra_res[xi] = be.extra_idx[xi];
                    ba.extra_pos[xi] = be.pos_of[be.extra_idx[xi]];
                    ba.invv[xi] = static_cast<int>(pmod(-be.invv[xi], be.moduli[be.extra_idx[xi]]));
                }
                ba.N = N;
                ba.n_tab = be.n_tab;
                ba.tab = upload_tables(li, "be");
                if (!be_work_) be_work_ = dalloc<int16_t>(static_cast<size_t>(B_) * k_ * 128 * maxN);
                ba.work = be_work_;
                ba.hard = hard_ ? 1 : 0;
                ba.gate0 = gate_base(li + 1, 1);
                add_op(lname, [ba, x, B, mc, ag](hipStream_t st) { launch_base_ext(ba, x, B, mc, ag, st); });
                break;
            }
            default:
                throw std::runtime_error(std::string("dash: HIP evaluator cannot run layer kind ") + kind_name(g.kind));
        }
        save_if_needed(li + 1, cur, N, mods);
    }
    if (stream_) add_op("stage_end", [this](hipStream_t st) { stage_end(st); });
    final_ = act_of(cur);
    Nout_ = N;
    out_mod_ = mods;
    for (int j = 0; j < k_; ++j) {
        act_t* p = nullptr;
        HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&p), sizeof(act_t) * B_ * nr_comps(mods[j]) * std::max<i64>(Nout_, 1)));
        host_allocs_.push_back(p);
        out_stage_.push_back(p);
        void* dp = nullptr;
        if (hipHostGetDevicePointer(&dp, p, 0) != hipSuccess || !dp) {
            (void)hipGetLastError();
            out_stage_mapped_ = false;
        }
        out_stage_dev_.push_back(dp);
    }
    finish_small();
    HIPCHECK(hipDeviceSynchronize());
}

void HipEvaluator::plan_rescale_legacy(size_t li, i64 iters, i64 N, const CrtInfo& crt, const std::string& lname) {
    const GarbledModel& m0 = *tmpl_;
    Act x = act_of(0);
    // the current activation buffer is whatever `cur` is; callers keep the
    // in-place convention: rescale always operates on the current buffer
    x = cur_act_;
    const ModC* mc = mc_;
    const AesGlobals ag = aes_;
    const int B = B_;
    const int ls = lab_stride_;
    DASH_CHECK(crt_[0] == 2, "legacy rescale needs crt[0] == 2");
    // per-GC constants: delta = up - down (all residues), du = bits(up0) ^ bits(down0)
    const int16_t* delta = nullptr;
    const u128* du = nullptr;
    {
        int16_t* dd = dalloc<int16_t>(static_cast<size_t>(B_) * lab_stride_);
        u128* ddu = dalloc<u128>(B_);
        const int k = k_;
        std::vector<int> off(lab_off_, lab_off_ + k_), crtv = crt_;
        add_small(reinterpret_cast<uint8_t*>(dd), sizeof(int16_t) * ls, sizeof(int16_t) * ls,
                  [ls, k, off, crtv](const GarbledModel& m, uint8_t* hb) {
            int16_t* h = reinterpret_cast<int16_t*>(hb);
            std::fill(h, h + ls, int16_t(0));
            for (int j = 0; j < k; ++j) {
                const int p = crtv[j], n = nr_comps(p);
                const int16_t* up = m.consts.at("up." + std::to_string(j)).ptr<int16_t>();
                const int16_t* dn = m.consts.at("down.2." + std::to_string(j)).ptr<int16_t>();
                for (int c = 0; c < n; ++c) h[off[j] + c] = static_cast<int16_t>(pmod(up[c] - dn[c], p));
            }
        });
        add_small(reinterpret_cast<uint8_t*>(ddu), sizeof(u128), sizeof(u128), [](const GarbledModel& m, uint8_t* hb) {
            u128 pk = 0;
            const int n = nr_comps(2);
            const int16_t* up = m.consts.at("up.0").ptr<int16_t>();
            const int16_t* dn = m.consts.at("down.2.0").ptr<int16_t>();
            for (int c = 0; c < n; ++c) pk |= static_cast<u128>((up[c] ^ dn[c]) & 1) << c;
            std::memcpy(hb, &pk, sizeof(u128));
        });
        delta = dd;
        du = ddu;
    }
    const int16_t* down = upload_const_rows([&](int j) { return "down.2." + std::to_string(j); });
    for (i64 it = 0; it < iters; ++it) {
        RescalePlan P(crt_, m0.h.mrs, {2}, true, m0.h.sign_fused != 0);
        const std::string pre = arr_name("it", static_cast<int>(it), ".");
        const u128* trans = upload_tables(li, pre + "trans");
        SignArgs sa = make_sign(li, pre, P.sign, N, 0);
        const int maxn = sign_maxn_;
        u128* h0 = h0_;
        uint16_t* col0 = col0_;
        if (it == 0) {
            const int16_t* up = up_rows_ + lab_off_[0];
            add_op(lname + ".hash", [x, up, ls, N, B, h0, col0, mc, ag](hipStream_t st) {
                launch_rescale_hash(x, 0, 2, up, ls, 1, N, B, h0, col0, mc, ag, st);
            });
        } else {
            const u128* sp = outP_;
            add_op(lname + ".hash", [sp, du, N, B, h0, col0, ag](hipStream_t st) {
                launch_rescale_hash_sign(sp, du, N, B, h0, col0, ag, st);
            });
        }
        RescaleArgs ra{};
        ra.crt = crt;
        ra.N = N;
        ra.fi = 0;
        ra.s = 2;
        ra.add_up = 1;
        for (size_t q = 0; q < P.active[0].size(); ++q) {
            const int jj = P.active[0][q];
            ra.active[jj] = 1;
            ra.aidx[jj] = static_cast<int>(q);
            ra.inv[jj] = static_cast<int>(P.inv[0][q]);
        }
        ra.n_trans = P.n_trans;
        ra.off = 0;
        ra.trans = trans;
        ra.h0 = h0_;
        ra.col0 = col0_;
        ra.lab_stride = lab_stride_;
        for (int j = 0; j < k_; ++j) ra.lab_off[j] = lab_off_[j];
        const int16_t* dl = it == 0 ? up_rows_ : delta;
        const u128* zh = zh_;
        add_op(lname + ".upd+A", [ra, sa, x, dl, zh, B, mc, ag](hipStream_t st) {
            launch_rescale_update_approx(ra, sa, x, dl, zh, B, mc, ag, st);
        });
        add_op(lname + ".B", [sa, maxn, mc, ag](hipStream_t st) { launch_sign_chain(sa, maxn, mc, ag, st); });
    }
    const u128* signP = outP_;
    const int* loff = d_lab_off_;
    add_op(lname + ".post", [x, crt, N, B, signP, down, ls, loff, mc](hipStream_t st) {
        launch_rescale_post(x, crt, N, B, signP, down, ls, loff, mc, st);
    });
}

// ---------------------------------------------------------------------------
// Garbler side of online message #1 on the device. The garbler's secrets for a GC's inputs (the base labels W0
// and the offsets R_p) are placed on the evaluator's GPU once, offline; encode then writes the encoded input
// W0 + x R straight into an evaluator slot's input activations (k_encode_in): only the plaintext input (8 B per
// element) crosses PCIe, and neither side compresses, stages or decompresses a label. This is the in-process form
// of the same-node device transport (IpcTables): the write target is the evaluator's, the labels are the
// garbler's, and the evaluator never reads W0 or R. An encoder holds `slots` GCs (one per evaluator slot of a
// group): encode_all writes all of them with one H2D and one launch.
class DeviceInputEncoder {
   public:
    // g arms encoder slot `slot` (the evaluator slot its tables went to); every other slot stays empty until
    // load() arms it with its own GC (encode refuses empty slots)
    DeviceInputEncoder(const Garbler& g, int device, int slots, int slot = 0)
        : dev_(device), S_(slots), crt_(g.crt()) {
        const CrtLabels& W0 = g.input_base();
        DASH_CHECK(S_ >= 1, "DeviceInputEncoder: slots must be >= 1");
        DASH_CHECK(!W0.empty() && W0.size() == crt_.size(), "DeviceInputEncoder: garble() must run first");
        DASH_CHECK(static_cast<int>(crt_.size()) <= kMaxRes, "DeviceInputEncoder: too many residues");
        bind_device(dev_, nullptr, "DeviceInputEncoder");
        N_ = W0[0].N;
        DASH_CHECK(N_ * 128 < (i64(1) << 31), "DeviceInputEncoder: input too large for the 32-bit lane index");
        a_.k = static_cast<int>(crt_.size());
        size_t off = 0;
        for (size_t j = 0; j < crt_.size(); ++j) {
            const Labels& L = W0[j];
            DASH_CHECK(L.p <= kActMaxModulus, "DeviceInputEncoder: modulus above the byte activations");
            a_.p[j] = L.p;
            a_.n[j] = L.n;
            w_off_.push_back(off);
            off += static_cast<size_t>(L.n) * N_;
            r_off_.push_back(off);
            off += L.n;
        }
        bytes_ = (off + 15) & ~size_t(15);
        a_.wstride = static_cast<int64_t>(bytes_);
        HIPCHECK(hipMalloc(reinterpret_cast<void**>(&w_), bytes_ * S_));
        HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&w_h_), bytes_));
        for (size_t j = 0; j < crt_.size(); ++j) {
            a_.w0[j] = w_ + w_off_[j];
            a_.r[j] = w_ + r_off_[j];
        }
        HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&x_h_), sizeof(int64_t) * N_ * S_));
        HIPCHECK(hipMalloc(reinterpret_cast<void**>(&x_d_), sizeof(int64_t) * N_ * S_));
        HIPCHECK(hipEventCreateWithFlags(&done_, hipEventDisableTiming));
        HIPCHECK(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
        loaded_.assign(S_, 0);
        load(g, slot);
    }
    ~DeviceInputEncoder() {
        (void)hipSetDevice(dev_);
        if (pending_) (void)hipEventSynchronize(done_);
        (void)hipStreamSynchronize(st_);
        (void)hipStreamDestroy(st_);
        (void)hipEventDestroy(done_);
        (void)hipFree(w_);
        (void)hipFree(x_d_);
        (void)hipHostFree(x_h_);
        (void)hipHostFree(w_h_);
        // teardown errors are ignored (e.g. done_'s last stream capturing in another thread): clear the thread's
        // last error so a later, unrelated HIPCHECK(hipGetLastError()) does not report it
        (void)hipGetLastError();
    }
    DeviceInputEncoder(const DeviceInputEncoder&) = delete;
    DeviceInputEncoder& operator=(const DeviceInputEncoder&) = delete;
    i64 input_size() const { return N_; }
    int slots() const { return S_; }
    // (re-)arm slot s with GC g of the same circuit and base (a serving slot's next GC): its base labels and
    // offsets replace the slot's current ones once the last encode has read them (synchronous, private stream).
    // Concurrent loads of different slots serialize on the shared host staging.
    void load(const Garbler& g, int s) {
        const CrtLabels& W0 = g.input_base();
        DASH_CHECK(s >= 0 && s < S_, "DeviceInputEncoder: slot out of range");
        DASH_CHECK(g.crt() == crt_ && !W0.empty() && W0[0].N == N_, "DeviceInputEncoder: another circuit or base");
        std::lock_guard<std::mutex> lk(load_mu_);
        bind_device(dev_, nullptr, "DeviceInputEncoder.load");
        if (pending_) HIPCHECK(hipEventSynchronize(done_));
        for (size_t j = 0; j < crt_.size(); ++j) {
            const Labels& L = W0[j];
            const comp_t* R = g.offsets().get(L.p);
            act_t* w = w_h_ + w_off_[j];
            for (i64 e = 0; e < N_; ++e)
                for (int c = 0; c < L.n; ++c) w[static_cast<size_t>(c) * N_ + e] = static_cast<act_t>(L.c[e * L.n + c]);
            for (int c = 0; c < L.n; ++c) w_h_[r_off_[j] + c] = static_cast<act_t>(R[c]);
        }
        HIPCHECK(hipMemcpyAsync(w_ + bytes_ * s, w_h_, bytes_, hipMemcpyHostToDevice, st_));
        HIPCHECK(hipStreamSynchronize(st_));
        loaded_[s] = 1;
    }
    // slots [0, n) <- x[n][N] into evaluator slots b0 .. b0 + n - 1, async on st (ordered before h.run on st)
    void encode(HipEvaluator& h, int b0, const i64* x, int n, i64 N, hipStream_t st) {
        DASH_CHECK(N == N_ && h.input_size() == N_, "DeviceInputEncoder: input size mismatch");
        DASH_CHECK(n >= 1 && n <= S_ && b0 >= 0 && b0 + n <= h.batch(), "DeviceInputEncoder: slot range mismatch");
        DASH_CHECK(h.crt() == crt_, "DeviceInputEncoder: the evaluator's CRT base differs from the garbler's");
        DASH_CHECK(h.device() == dev_, "DeviceInputEncoder: the evaluator lives on another device");
        for (int s = 0; s < n; ++s) DASH_CHECK(loaded_[s], "DeviceInputEncoder: slot " + std::to_string(s) + " has no GC");
        bind_device(dev_, st, "DeviceInputEncoder.encode");
        if (pending_) HIPCHECK(hipEventSynchronize(done_));  // the previous H2D has read the pinned staging
        std::memcpy(x_h_, x, sizeof(int64_t) * N_ * n);
        HIPCHECK(hipMemcpyAsync(x_d_, x_h_, sizeof(int64_t) * N_ * n, hipMemcpyHostToDevice, st));
        EncIn a = a_;
        for (int j = 0; j < a.k; ++j) a.out[j] = h.input_act(b0, j);
        launch_encode_in(a, x_d_, N_, n, st);
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipEventRecord(done_, st));
        pending_ = true;
    }

   private:
    int dev_, S_;
    std::vector<int> crt_;
    i64 N_ = 0;
    EncIn a_{};
    std::vector<size_t> w_off_, r_off_;
    std::vector<int> loaded_;
    size_t bytes_ = 0;
    act_t* w_ = nullptr;
    act_t* w_h_ = nullptr;
    hipStream_t st_ = nullptr;
    std::mutex load_mu_;
    int64_t* x_h_ = nullptr;
    int64_t* x_d_ = nullptr;
    hipEvent_t done_ = nullptr;
    bool pending_ = false;
};

// ---------------------------------------------------------------------------
namespace {
py::list labels_to_py2(const CrtLabels& L) {
    py::list out;
    for (const auto& x : L) {
        py::array_t<int16_t> arr({static_cast<py::ssize_t>(x.N), static_cast<py::ssize_t>(x.n)});
        std::memcpy(arr.mutable_data(), x.c.data(), x.c.size() * sizeof(comp_t));
        out.append(py::make_tuple(x.p, arr));
    }
    return out;
}
CrtLabels labels_from_py2(const py::list& l) {
    CrtLabels out;
    for (auto item : l) {
        py::tuple t = item.cast<py::tuple>();
        int p = t[0].cast<int>();
        auto arr = py::array_t<int16_t, py::array::c_style | py::array::forcecast>::ensure(t[1]);
        DASH_CHECK(arr && arr.ndim() == 2, "labels must be (N, n) int16 arrays");
        Labels L(p, arr.shape(0));
        DASH_CHECK(arr.shape(1) == L.n, "label width does not match modulus");
        std::memcpy(L.c.data(), arr.data(), L.c.size() * sizeof(comp_t));
        out.push_back(std::move(L));
    }
    return out;
}
hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }
}  // namespace

void register_guard_bindings(py::module_& m);  // guard.hip

void register_hip_bindings(py::module_& m) {
    register_guard_bindings(m);
    m.def("encode_compressed_into", [](const Garbler& g, py::array_t<i64, py::array::c_style | py::array::forcecast> x,
                                       HipEvaluator& h, int b) {
        DASH_CHECK(x.size() == h.input_size(), "input size mismatch");
        u128* dst = h.input_slot_compressed(b);
        const i64* xp = x.data();
        const i64 N = x.size();
        py::gil_scoped_release rel;
        g.encode_compressed(xp, N, dst);
    });
    py::class_<DeviceInputEncoder>(m, "DeviceInputEncoder")
        .def(py::init<const Garbler&, int, int, int>(), py::arg("garbler"), py::arg("device"), py::arg("slots") = 1,
             py::arg("slot") = 0)
        .def("input_size", &DeviceInputEncoder::input_size)
        .def("slots", &DeviceInputEncoder::slots)
        .def("load", &DeviceInputEncoder::load, py::arg("garbler"), py::arg("slot") = 0,
             py::call_guard<py::gil_scoped_release>())
        // x: (N,) for one slot or (n, N) for slots 0 .. n - 1 -> evaluator slots b0 ..
        .def("encode_into", [](DeviceInputEncoder& enc, HipEvaluator& h, int b0,
                               py::array_t<i64, py::array::c_style | py::array::forcecast> x, uintptr_t stream) {
            const int n = x.ndim() == 2 ? static_cast<int>(x.shape(0)) : 1;
            const i64 N = x.ndim() == 2 ? static_cast<i64>(x.shape(1)) : static_cast<i64>(x.size());
            DASH_CHECK(x.ndim() == 1 || x.ndim() == 2, "DeviceInputEncoder: x must be (N,) or (slots, N)");
            enc.encode(h, b0, x.data(), n, N, as_stream(stream));
        }, py::arg("evaluator"), py::arg("slot"), py::arg("x"), py::arg("stream") = 0);
    // in-process two-party fast path: the garbler encodes straight into the
    // evaluator's pinned staging slot (the bytes are exactly online message #1)
    m.def("encode_into", [](const Garbler& g, py::array_t<i64, py::array::c_style | py::array::forcecast> x,
                            HipEvaluator& h, int b) {
        auto slot = h.input_slot(b);
        DASH_CHECK(x.size() == h.input_size(), "input size mismatch");
        const i64* xp = x.data();
        const i64 N = x.size();
        py::gil_scoped_release rel;
        g.encode_cm(xp, N, slot);
    });
    // Dedicated non-blocking HIP streams (each new stream is mapped to the next
    // hardware queue), for running independent GC groups concurrently.
    m.def("hip_stream_create", [](int priority) {
        hipStream_t st = nullptr;
        HIPCHECK(hipStreamCreateWithPriority(&st, hipStreamNonBlocking, priority));
        return reinterpret_cast<uintptr_t>(st);
    }, py::arg("priority") = 0);
    m.def("hip_stream_destroy", [](uintptr_t st) { HIPCHECK(hipStreamDestroy(reinterpret_cast<hipStream_t>(st))); });
    m.def("hip_stream_sync", [](uintptr_t st) { HIPCHECK(hipStreamSynchronize(reinterpret_cast<hipStream_t>(st))); });
    // Watchdog primitive: wait for a stream with a deadline instead of an
    // unbounded hipStreamSynchronize (which a hung kernel never returns from).
    // Polls hipStreamQuery with the GIL released; true = drained, false = the
    // deadline passed with work still queued. Errors raised by the stream throw.
    m.def("hip_stream_wait", [](uintptr_t st, double timeout_s) {
        py::gil_scoped_release rel;
        const auto t0 = std::chrono::steady_clock::now();
        for (int spin = 0;; ++spin) {
            const hipError_t e = hipStreamQuery(reinterpret_cast<hipStream_t>(st));
            if (e == hipSuccess) return true;
            if (e != hipErrorNotReady) HIPCHECK(e);
            const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (timeout_s >= 0 && dt > timeout_s) return false;
            if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(spin > 4096 ? 1000 : 50));
        }
    }, py::arg("stream"), py::arg("timeout_s"));
    // Reset the thread's sticky last-error (e.g. after a handled out-of-memory), so a later
    // hipGetLastError() launch check does not report it again. Returns the cleared code.
    m.def("hip_clear_last_error", []() { return static_cast<int>(hipGetLastError()); });
    m.def("hip_device_count", []() {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) return 0;
        return n;
    });
    // "dddd:bb:dd.f" of a device (multi-GPU bench evidence: which physical GPU each rank ran on)
    m.def("hip_device_pci_bus_id", [](int device) {
        char buf[64] = {0};
        HIPCHECK(hipDeviceGetPCIBusId(buf, static_cast<int>(sizeof(buf)), device));
        return std::string(buf);
    });
    py::class_<IpcTables, std::shared_ptr<IpcTables>>(m, "IpcTables")
        .def(py::init([](int device, const py::list& handles, int B) {
                 std::vector<std::tuple<size_t, std::string, size_t, std::string>> hs;
                 for (auto item : handles) {
                     auto t = item.cast<py::tuple>();
                     hs.emplace_back(t[0].cast<size_t>(), t[1].cast<std::string>(), t[2].cast<size_t>(),
                                     t[3].cast<std::string>());
                 }
                 return std::make_shared<IpcTables>(device, hs, B);
             }),
             py::arg("device"), py::arg("handles"), py::arg("batch"))
        .def("tables", &IpcTables::tables)
        .def("sink", &IpcTables::sink, "slot b of the evaluator's table arenas as a GPU-garbler destination");
    py::class_<HipEvaluator, std::shared_ptr<HipEvaluator>>(m, "HipEvaluator")
        .def(py::init([](std::shared_ptr<GarbledModel> tmpl, int B, int device, bool mfma, bool stream_tables) {
                 return std::make_shared<HipEvaluator>(std::move(tmpl), B, device, mfma, stream_tables);
             }),
             py::arg("template"), py::arg("batch"), py::arg("device") = 0, py::arg("mfma") = true,
             py::arg("stream_tables") = false)
        .def_property_readonly("streams_tables", &HipEvaluator::streams_tables)
        .def("load", [](HipEvaluator& h, int b, std::shared_ptr<GarbledModel> m) {
            py::gil_scoped_release rel;
            h.load(b, *m);
        })
        .def("sink", &HipEvaluator::sink, "slot b's table arenas as a GPU-garbler destination (zero-copy load)")
        .def("ipc_export", [](const HipEvaluator& h) {
            py::list out;
            for (const auto& e : h.ipc_export())
                out.append(py::make_tuple(std::get<0>(e), std::get<1>(e), std::get<2>(e), py::bytes(std::get<3>(e))));
            return out;
        }, "IPC handles of the table arenas: [(layer, table, bytes per slot, handle)] (same-node device transport)")
        .def_property_readonly("batch", &HipEvaluator::batch)
        .def("device_bytes", &HipEvaluator::device_bytes)
        .def("table_bytes", &HipEvaluator::table_bytes)
        .def("set_profile", &HipEvaluator::set_profile)
        .def("op_times", &HipEvaluator::op_times)
        .def("set_inputs", [](HipEvaluator& h, const py::list& inputs, uintptr_t stream) {
            std::vector<CrtLabels> in;
            for (auto it : inputs) in.push_back(labels_from_py2(it.cast<py::list>()));
            h.set_inputs(in, as_stream(stream));
        }, py::arg("inputs"), py::arg("stream") = 0)
        .def("run", [](HipEvaluator& h, uintptr_t stream) { h.run(as_stream(stream)); }, py::arg("stream") = 0)
        .def("set_input_cm", [](HipEvaluator& h, int b, const py::list& arrs) {
            auto slot = h.input_slot(b);
            DASH_CHECK(static_cast<size_t>(py::len(arrs)) == slot.size(), "one array per residue expected");
            for (size_t j = 0; j < slot.size(); ++j) {
                auto a = py::array_t<int16_t, py::array::c_style | py::array::forcecast>::ensure(arrs[j]);
                std::memcpy(slot[j], a.data(), a.size() * sizeof(int16_t));
            }
        })
        .def("upload_inputs", [](HipEvaluator& h, uintptr_t stream) { h.upload_inputs(as_stream(stream)); }, py::arg("stream") = 0)
        .def("set_input_compressed", [](HipEvaluator& h, int b, py::array_t<uint64_t, py::array::c_style | py::array::forcecast> c) {
            DASH_CHECK(c.ndim() == 3 && c.shape(0) == h.crt_size() && c.shape(1) == h.input_size() && c.shape(2) == 2,
                       "compressed inputs must be (k, N, 2) uint64");
            std::memcpy(h.input_slot_compressed(b), c.data(), sizeof(u128) * h.crt_size() * h.input_size());
        })
        .def("upload_inputs_compressed", [](HipEvaluator& h, uintptr_t stream) { h.upload_inputs_compressed(as_stream(stream)); },
             py::arg("stream") = 0)
        .def("fetch_outputs", [](HipEvaluator& h, uintptr_t stream) { h.fetch_outputs(as_stream(stream)); }, py::arg("stream") = 0)
        .def("crt_size", &HipEvaluator::crt_size)
        .def("set_graph", &HipEvaluator::set_graph)
        .def("input_size", &HipEvaluator::input_size)
        .def("output_size", &HipEvaluator::output_size)
        .def("outputs_compressed", [](const HipEvaluator& h, int b) {
            auto r = h.outputs_compressed(b);
            py::array_t<uint64_t> out({static_cast<py::ssize_t>(h.crt_size()), static_cast<py::ssize_t>(h.output_size()),
                                       static_cast<py::ssize_t>(2)});
            std::memcpy(out.mutable_data(), r.data(), r.size() * sizeof(u128));
            return out;
        })
        .def("decode_into", [](const HipEvaluator& h, int b, const Decoder& d) {
            // online message #2 (compressed) decoded by the garbler, no Python round trip
            auto r = h.outputs_compressed(b);
            return d.decode_compressed(r.data());
        })
        .def("get_outputs", [](HipEvaluator& h, uintptr_t stream) {
            auto o = h.get_outputs(as_stream(stream));
            py::list r;
            for (auto& x : o) r.append(labels_to_py2(x));
            return r;
        }, py::arg("stream") = 0)
        .def("evaluate", [](HipEvaluator& h, const py::list& inputs, uintptr_t stream) {
            std::vector<CrtLabels> in;
            for (auto it : inputs) in.push_back(labels_from_py2(it.cast<py::list>()));
            std::vector<CrtLabels> o;
            {
                py::gil_scoped_release rel;
                h.set_inputs(in, as_stream(stream));
                h.run(as_stream(stream));
                o = h.get_outputs(as_stream(stream));
            }
            py::list r;
            for (auto& x : o) r.append(labels_to_py2(x));
            return r;
        }, py::arg("inputs"), py::arg("stream") = 0);

    // parity helpers for tests
    m.def("hip_aes_hash_array", [](py::array_t<uint64_t, py::array::c_style | py::array::forcecast> a) {
        DASH_CHECK(a.ndim() == 2 && a.shape(1) == 2, "expected (n,2) uint64");
        const int64_t n = a.shape(0);
        auto te = make_te0();
        auto rk = fixed_round_key_words();
        uint32_t *dte, *drk;
        u128 *din, *dout;
        HIPCHECK(hipMalloc(&dte, 256 * 4));
        HIPCHECK(hipMalloc(&drk, 44 * 4));
        HIPCHECK(hipMalloc(&din, n * 16 + 16));
        HIPCHECK(hipMalloc(&dout, n * 16 + 16));
        HIPCHECK(hipMemcpy(dte, te.data(), 256 * 4, hipMemcpyHostToDevice));
        HIPCHECK(hipMemcpy(drk, rk.data(), 44 * 4, hipMemcpyHostToDevice));
        HIPCHECK(hipMemcpy(din, a.data(), n * 16, hipMemcpyHostToDevice));
        AesGlobals g{dte, drk};
        launch_aes_test(din, dout, n, g, nullptr);
        py::array_t<uint64_t> out({static_cast<py::ssize_t>(n), static_cast<py::ssize_t>(2)});
        HIPCHECK(hipMemcpy(out.mutable_data(), dout, n * 16, hipMemcpyDeviceToHost));
        (void)hipFree(dte); (void)hipFree(drk); (void)hipFree(din); (void)hipFree(dout);
        return out;
    });
    m.def("hip_hard_pads", [](py::array_t<uint64_t, py::array::c_style | py::array::forcecast> keys,
                              py::array_t<uint64_t, py::array::c_style | py::array::forcecast> gates,
                              py::array_t<uint32_t, py::array::c_style | py::array::forcecast> subs,
                              py::array_t<uint32_t, py::array::c_style | py::array::forcecast> blks) {
        DASH_CHECK(keys.ndim() == 2 && keys.shape(1) == 2, "keys: (n, 2) uint64");
        const int64_t n = keys.shape(0);
        DASH_CHECK(gates.size() == n && subs.size() == n && blks.size() == n, "one gate / sub / block per key");
        u128 *dk, *dout;
        uint64_t* dg;
        uint32_t *ds, *db;
        HIPCHECK(hipMalloc(&dk, n * 16 + 16));
        HIPCHECK(hipMalloc(&dout, n * 64 + 64));
        HIPCHECK(hipMalloc(&dg, n * 8 + 8));
        HIPCHECK(hipMalloc(&ds, n * 4 + 4));
        HIPCHECK(hipMalloc(&db, n * 4 + 4));
        HIPCHECK(hipMemcpy(dk, keys.data(), n * 16, hipMemcpyHostToDevice));
        HIPCHECK(hipMemcpy(dg, gates.data(), n * 8, hipMemcpyHostToDevice));
        HIPCHECK(hipMemcpy(ds, subs.data(), n * 4, hipMemcpyHostToDevice));
        HIPCHECK(hipMemcpy(db, blks.data(), n * 4, hipMemcpyHostToDevice));
        launch_hard_test(dk, dg, ds, db, dout, n, nullptr);
        py::array_t<uint64_t> out({static_cast<py::ssize_t>(n), static_cast<py::ssize_t>(4), static_cast<py::ssize_t>(2)});
        HIPCHECK(hipMemcpy(out.mutable_data(), dout, n * 64, hipMemcpyDeviceToHost));
        (void)hipFree(dk); (void)hipFree(dout); (void)hipFree(dg); (void)hipFree(ds); (void)hipFree(db);
        return out;
    }, "hardened-encoding pads computed on the GPU (dev.h hard_block), (n, 4, 2) uint64");
    m.def("hip_aes_bench", [](int blocks, int iters) {
        // returns (ms, AES blocks per second)
        auto te = make_te0();
        uint32_t* dte;
        u128* dout;
        HIPCHECK(hipMalloc(&dte, 256 * 4));
        HIPCHECK(hipMalloc(&dout, static_cast<size_t>(blocks) * 512 * 16));
        HIPCHECK(hipMemcpy(dte, te.data(), 256 * 4, hipMemcpyHostToDevice));
        AesGlobals g{dte, nullptr};
        launch_aes_bench(dout, blocks, 4, g, nullptr);  // warm-up
        hipEvent_t e0, e1;
        HIPCHECK(hipEventCreate(&e0));
        HIPCHECK(hipEventCreate(&e1));
        HIPCHECK(hipEventRecord(e0, nullptr));
        launch_aes_bench(dout, blocks, iters, g, nullptr);
        HIPCHECK(hipEventRecord(e1, nullptr));
        HIPCHECK(hipEventSynchronize(e1));
        float ms = 0;
        HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
        (void)hipEventDestroy(e0); (void)hipEventDestroy(e1);
        (void)hipFree(dte); (void)hipFree(dout);
        const double n = 2.0 * iters * blocks * 512.0;
        return py::make_tuple(ms, n / (ms * 1e-3));
    });
    m.def("hip_codec", [](py::array_t<int16_t, py::array::c_style | py::array::forcecast> labels, int q) {
        // labels (N, n) label-major -> (compressed (N,2) u64, decompressed (N, n))
        DASH_CHECK(labels.ndim() == 2, "expected (N, n)");
        const int64_t N = labels.shape(0), n = labels.shape(1);
        DASH_CHECK(n == nr_comps(q), "label width mismatch");
        std::vector<int16_t> cm(N * n);
        for (int64_t e = 0; e < N; ++e)
            for (int64_t c = 0; c < n; ++c) cm[c * N + e] = labels.data()[e * n + c];
        std::vector<ModC> mc(q + 1);
        mc[q] = make_modc(q);
        ModC* dmc;
        int16_t *dl, *dd;
        u128* dc;
        HIPCHECK(hipMalloc(&dmc, sizeof(ModC) * (q + 1)));
        HIPCHECK(hipMalloc(&dl, N * n * 2));
        HIPCHECK(hipMalloc(&dd, N * n * 2));
        HIPCHECK(hipMalloc(&dc, N * 16));
        HIPCHECK(hipMemcpy(dmc, mc.data(), sizeof(ModC) * (q + 1), hipMemcpyHostToDevice));
        HIPCHECK(hipMemcpy(dl, cm.data(), N * n * 2, hipMemcpyHostToDevice));
        launch_codec_test(dl, N, q, dmc, dc, dd, nullptr);
        py::array_t<uint64_t> comp({static_cast<py::ssize_t>(N), static_cast<py::ssize_t>(2)});
        HIPCHECK(hipMemcpy(comp.mutable_data(), dc, N * 16, hipMemcpyDeviceToHost));
        std::vector<int16_t> dec(N * n);
        HIPCHECK(hipMemcpy(dec.data(), dd, N * n * 2, hipMemcpyDeviceToHost));
        py::array_t<int16_t> decomp({static_cast<py::ssize_t>(N), static_cast<py::ssize_t>(n)});
        for (int64_t e = 0; e < N; ++e)
            for (int64_t c = 0; c < n; ++c) decomp.mutable_data()[e * n + c] = dec[c * N + e];
        (void)hipFree(dmc); (void)hipFree(dl); (void)hipFree(dd); (void)hipFree(dc);
        return py::make_tuple(comp, decomp);
    });
}

}  // namespace dash
