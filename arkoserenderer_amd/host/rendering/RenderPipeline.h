// RenderPipeline.h — node list + construction/execution order (RenderPipeline.h:11-78,
// RenderPipeline.cpp:35-68: insertion order).
#pragma once

#include <memory>
#include <vector>

#include "RenderPipelineNode.h"

class RenderPipeline {
public:
    explicit RenderPipeline(GpuScene* scene) : m_scene(scene) {}

    RenderPipelineNode& addNode(std::unique_ptr<RenderPipelineNode>&& node);
    template<typename NodeType, typename... Args>
    NodeType& addNode(Args&&... args)
    {
        return static_cast<NodeType&>(addNode(std::make_unique<NodeType>(std::forward<Args>(args)...)));
    }

    void constructAll(Registry& registry);
    void forEachNodeInResolvedOrder(const std::function<void(RenderPipelineNode&, const RenderPipelineNode::ExecuteCallback&)>&) const;

    // Executes every node's callback for one frame on the backend's stream
    // (the headless "submit and wait" pattern of MeshViewerApp.cpp:845-893).
    void executeFrame(const AppState&, HipBackend&) const;

private:
    struct NodeContext {
        RenderPipelineNode* node;
        RenderPipelineNode::ExecuteCallback executeCallback;
    };
    GpuScene* m_scene;
    std::vector<std::unique_ptr<RenderPipelineNode>> m_ownedNodes;
    std::vector<NodeContext> m_nodeContexts;
};
