// RenderPipelineNode.h — node plugin interface (arkose/rendering/RenderPipelineNode.h:18-52).
#pragma once

#include <functional>
#include <string>

#include "AppState.h"
#include "Registry.h"
#include "backend/hip/HipBackend.h"

class GpuScene;

class RenderPipelineNode {
public:
    RenderPipelineNode() = default;
    virtual ~RenderPipelineNode() = default;

    using ExecuteCallback = std::function<void(const AppState&, CommandList&, UploadBuffer&)>;

    // An execute callback that does nothing (RenderPipelineNode.cpp:8).
    static const ExecuteCallback NullExecuteCallback;

    virtual std::string name() const = 0;
    virtual ExecuteCallback construct(GpuScene&, Registry&) = 0;
    virtual void drawGui() {}
};
